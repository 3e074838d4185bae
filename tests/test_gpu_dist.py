"""World-2 data-parallel trainer step on the GPU box's one card (two ranks on cuda:0, gloo): the overlapped bucketed
gradient all-reduce equals the flat one, the synced gradient and the post-step LoRA masters are identical on both
ranks (tests/dist_worker_gpu.py).  The ranks run as child processes of torch.distributed.run."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]
HERE = os.path.dirname(os.path.abspath(__file__))


def test_world2_trainer_step_bucketed_overlap(tmp_path):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.join(HERE, "dist_worker_gpu.py"), "--out", str(tmp_path)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = [json.load(open(os.path.join(tmp_path, f"rank{i}.json"))) for i in range(2)]
    print(res)
    for d in res:
        assert d["armed"] and d["buckets"] >= 3
        assert d["issued_before_finish"] == d["buckets"]  # every bucket left during the backward
        assert d["scale"] == 0.5
        assert d["grad_norm"] > 0
        assert d["bucketed_vs_flat_rel"] < 1e-5           # float-atomic rounding of the dW kernels only
        assert d["synced_equal_across_ranks"] and d["masters_equal_across_ranks"]
