"""world_size-2 gloo runs of the data-parallel host logic (the N>1 path of bench.py / the trainer) on CPU:
gradient bucket sync + mean folding, max-over-ranks step timing, per-rank seeding."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from pairwise_sample_optimization_amd.trainer import allreduce_grads
        from bench import max_over_ranks
        torch.manual_seed(rank)                      # bench.py / T:238 device_specific seeding
        g = torch.randn(1000)
        local = g.clone()
        scale = allreduce_grads(g)
        allg = [torch.empty_like(local) for _ in range(world)]
        dist.all_gather(allg, local)
        mean = torch.stack(allg).mean(0)
        ok_mean = torch.allclose(g * scale, mean, rtol=1e-6, atol=1e-7)
        distinct = not torch.equal(allg[0], allg[1])
        t = max_over_ranks(0.5 + rank, None)
        q.put((rank, ok_mean, distinct, scale, t))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_gloo_world2_grad_sync_and_timing():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=100) for _ in range(world)]
    for p in procs:
        p.join(30)
        assert p.exitcode == 0
    for rank, ok_mean, distinct, scale, t in res:
        assert ok_mean and distinct
        assert scale == 0.5
        assert t == 1.5


def test_single_process_sync_is_identity():
    from pairwise_sample_optimization_amd.trainer import allreduce_grads
    g = torch.ones(3)
    assert allreduce_grads(g) == 1.0 and torch.equal(g, torch.ones(3))
