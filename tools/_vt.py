"""Run the given pytest node ids with an attention-variant knob set first (A/B of numerics-sensitive tests)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pytest
from pairwise_sample_optimization_amd import kernels as K

K.lib().pso_attention_set_variant(int(sys.argv[1]))
sys.exit(pytest.main(["-q", "-s", "-p", "no:cacheprovider"] + sys.argv[2:]))
