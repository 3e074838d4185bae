import os, sys
os.environ.setdefault("PSO_LIB", "knobs")  # benchmark knobs: the tools build (include/pso_amd_knobs.h)
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from pairwise_sample_optimization_amd import kernels as K
K.gemm_set_variant(int(os.environ["V"]))
import pytest
sys.exit(pytest.main(["-x", "-q", "--timeout", "200", "--timeout-method", "thread", "tests/test_gpu_trainer.py", "-k", "graph_epoch_equals_eager"]))
