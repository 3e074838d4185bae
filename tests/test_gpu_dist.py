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
        assert d["bucketed_vs_flat_rel"] == 0.0           # every reduction is ordered: same bits either way
        assert d["synced_equal_across_ranks"] and d["masters_equal_across_ranks"]


def test_world2_full_unet_step_bf16_wire(tmp_path):
    """The C4 data-parallel step (full-UNet grads, frozen reference UNet, per-tensor 8-bit AdamW, bf16 wire) at world
    2: bucketed == flat on the same local gradient bit for bit, the local gradient bit-reproducible and the
    overlapped sync equal to the flat one bit for bit (no float atomics left in the backward), equal ranks after the
    optimizer step, and a zero gradient buffer after it
    (tests/dist_worker_gpu.py --full)."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.join(HERE, "dist_worker_gpu.py"), "--out", str(tmp_path),
           "--full"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = [json.load(open(os.path.join(tmp_path, f"rank{i}.json"))) for i in range(2)]
    print(res)
    for d in res:
        assert d["armed"] and d["buckets"] >= 3
        assert d["issued_before_finish"] == d["buckets"]
        assert d["wire"] == "torch.bfloat16" and d["scale"] == 0.5
        assert d["grad_norm"] > 0
        assert d["bucketed_equals_flat"]
        # every sum of the full-UNet backward is ordered (no float atomics): the local gradient is bit-reproducible,
        # so the sync overlapped with the backward equals the flat sync bit for bit, bf16 wire included
        assert d["local_run_to_run_equal"]
        assert d["overlapped_equals_flat"] and d["overlapped_vs_flat_rel"] == 0.0
        assert d["synced_equal_across_ranks"] and d["masters_equal_across_ranks"] and d["work_equal_across_ranks"]
        assert d["weights_moved"]
        assert d["grad_max_after_step"] == 0.0


def test_rccl_world1_bucketed_overlap_on_comm_stream(tmp_path):
    """The product's RCCL path (init_process_group("nccl"), bench.py's backend) on the box's one GPU at world size 1:
    RCCL still runs every collective on its own stream, so this exercises what the gloo tests cannot -- side.join()
    before each async all_reduce with the side-stream LoRA dW kernels still in flight, work.wait() as a stream wait in
    finish(), the bf16 wire cast back -- against the flat sync, bit for bit (tests/rccl_worker_gpu.py)."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1", "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.join(HERE, "rccl_worker_gpu.py"), "--out", str(tmp_path)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    d = json.load(open(os.path.join(tmp_path, "rank0.json")))
    print(d)
    assert d["backend"] == "nccl" and d["world"] == 1
    assert d["buckets"] >= 8 and d["issued_before_finish"] == d["buckets"]
    assert d["side_pending_at_issue"] > 0              # dW kernels were in flight on the side stream at some issue
    assert d["grad_norm"] > 0
    assert d["bucketed_equals_flat"] and d["wire_bf16_equals_cast"] and d["masters_equal"]
