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


def _bucket_worker(rank, world, port, q, wire=None):
    """GradBuckets on a fake 5-unit backward: buckets fire as their last unit completes, in completion order, and
    the bucketed sum equals the flat all-reduce (bf16 wire: within the bf16 rounding of the two summands and the
    sum, and every element is the bf16 sum cast back)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from pairwise_sample_optimization_amd.trainer import GradBuckets
        units = [("u0", 0, 300), ("u1", 300, 100), ("u2", 400, 500), ("u3", 900, 50), ("u4", 950, 74)]

        class FakeUNet:
            def grad_unit_ranges(self):
                return units

        torch.manual_seed(10 + rank)
        flat = torch.randn(1024)
        expect = flat.clone()
        dist.all_reduce(expect)
        gb = GradBuckets(FakeUNet(), flat, bucket_mb=400 * 4 / 1e6, wire_dtype=wire)   # 400-element buckets
        spans = [(o, n) for o, n, _ in gb.buckets]
        rt = type("RT", (), {})()
        done = gb.hook(rt)
        issued = []
        for u, _, _ in units:
            done(u)
            issued.append(sum(w is not None for w in gb.works))
        scale = gb.finish()
        if wire is None:
            ok = torch.equal(flat, expect)
        else:
            # bf16 rounding of the summands and of the sum (per element relative to the summands, so cancelling sums
            # can be far off relatively): rel-L2 over the vector
            ok = ((flat - expect).norm() / expect.norm()).item() < 1e-2 and torch.equal(flat, flat.to(wire).float())
            assert gb.bytes_on_wire() == 1024 * 2
        q.put((rank, spans, issued, ok, scale))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(120)
@pytest.mark.parametrize("wire", [None, torch.bfloat16])
def test_gloo_world2_bucketed_overlap_sync(wire):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_bucket_worker, args=(r, world, port, q, wire)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=100) for _ in range(world)]
    for p in procs:
        p.join(30)
        assert p.exitcode == 0
    for rank, spans, issued, equal, scale in res:
        assert spans == [(0, 400), (400, 500), (900, 124)]   # contiguous, completion-ordered buckets
        assert issued == [0, 1, 2, 2, 3]                      # each fires with its last unit, not at the end
        assert equal and scale == 0.5


@pytest.mark.parametrize("full", [False, True])
def test_grad_units_tile_the_flat_gradient(full):
    """The backward's unit order (UNet2DConditionModel.grad_units) tiles the trained flat gradient contiguously --
    the LoRA layout (reverse forward order of blocks) and the full-UNet layout (ordered by grad_units) -- so every
    all-reduce bucket is final when it is issued.  Host-only (CPU tensors, no kernel runs)."""
    from types import SimpleNamespace
    from pairwise_sample_optimization_amd.unet import UNet2DConditionModel, UNetConfig
    unet = UNet2DConditionModel(UNetConfig.tiny(16))
    if full:
        fg = unet.enable_full_grads()
        n = fg.numel
        slot = lambda k: -(-k // fg.ALIGN) * fg.ALIGN  # every tensor on a 64-element slot boundary
        assert n == sum(slot(p.numel()) for p in unet.parameters())
        assert all(off % fg.ALIGN == 0 for off, _ in fg.offsets.values())
    else:
        st = unet.add_adapter(SimpleNamespace(r=8, lora_alpha=8))
        n = st.numel
    ranges = unet.grad_unit_ranges()
    assert ranges[0][1] == 0 and sum(k for _, _, k in ranges) == n
    names = [u for u, _, _ in ranges]
    assert len(names) == len(set(names))
    if full:
        assert names[0] == "conv_out" and names[-1] == "embed"
    else:
        assert names[0].startswith("up_blocks.1.attentions") and names[-1] == "down_blocks.1.attentions.0"


def test_single_process_sync_is_identity():
    from pairwise_sample_optimization_amd.trainer import allreduce_grads
    g = torch.ones(3)
    assert allreduce_grads(g) == 1.0 and torch.equal(g, torch.ones(3))


def _flat_bf16_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from pairwise_sample_optimization_amd.trainer import allreduce_grads
        torch.manual_seed(rank)
        g = torch.randn(777)
        expect = g.clone()
        dist.all_reduce(expect)
        scale = allreduce_grads(g, wire_dtype=torch.bfloat16)
        q.put((scale, ((g - expect).norm() / expect.norm()).item() < 1e-2, g.dtype == torch.float32))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_gloo_world2_flat_allreduce_bf16_wire():
    """The un-bucketed sync (hipGraph epochs) with a bf16 wire: fp32 gradient in, fp32 sum out, bf16-close."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_flat_bf16_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=100) for _ in range(world)]
    for p in procs:
        p.join(30)
        assert p.exitcode == 0
    for scale, close, f32 in res:
        assert scale == 0.5 and close and f32
