"""Bit-exact determinism of the forward path (VERDICT r2 "what's weak" #2).

The forward of the paired UNet pass has no float atomics (split-K atomics only appear in the weight-gradient TN
products of the backward), so the same inputs must give the same bits whether the kernels are launched eagerly or
replayed from a captured hipGraph, run after run.  These tests pin that, for:
  * the flash-attention forward alone (self-attention at the 64^2 / 32^2 levels, cross-attention over 77 tokens, and
    an input that forces the rescale branch mid-row), for both row-max forms: the shipped one and the lane-local
    growth test (attention variant 1, the round-2 commit ea590ae that was reverted on suspicion of a hazard) -- they
    must also agree with each other bit for bit (same decisions, same arithmetic);
  * the whole paired SDXL UNet forward at 1024^2 (policy + reference images in one pass), eager vs graph replay;
  * the trainer's hipGraph epoch with the fp8 forward on (the captured graph must re-quantise the LoRA
    B stacks after every optimizer step, not replay the capture-time copies) -- now bit for bit: the LoRA weight
    gradients are reduced in a fixed order (no float atomics left on the LoRA training path);
  * the LoRA backward with its weight-gradient closures on the side stream vs in line.
"""
from types import SimpleNamespace

import pytest
import torch

from pairwise_sample_optimization_amd import _lib

pytestmark = pytest.mark.gpu


def _attn_inputs(cuda, B, H, Sq, Sk, seed, spike=False):
    g = torch.Generator(device="cuda").manual_seed(seed)
    C = H * 64
    q = torch.randn(B, Sq, C, device=cuda, generator=g).bfloat16()
    k = torch.randn(B, Sk, C, device=cuda, generator=g).bfloat16()
    v = torch.randn(B, Sk, C, device=cuda, generator=g).bfloat16()
    if spike:  # one key far above the rest, late in the row: the running max jumps past the rescale threshold there
        k[:, Sk - 70] = q[:, 5] * 6.0
    return q, k, v


def _run_variant(K, variant, fn):
    if variant == 0 and not _lib.KNOBS:  # the product library runs the default forms (no knobs)
        return fn()
    K.lib().pso_attention_set_variant(variant)
    try:
        return fn()
    finally:
        K.lib().pso_attention_set_variant(0)


def _variants(*vs):
    """The default form (0) everywhere; the knob-pinned forms in the tools build (PSO_LIB=knobs child process)."""
    return vs if _lib.KNOBS else (0,)


@pytest.mark.knob_variants
@pytest.mark.parametrize("shape", [(4, 10, 4096, 4096), (16, 20, 1024, 1024), (4, 10, 4096, 77), (2, 20, 1000, 77)])
@pytest.mark.parametrize("spike", [False, True])
def test_attention_fwd_bit_deterministic_eager_and_graph(cuda, shape, spike):
    from pairwise_sample_optimization_amd import kernels as K
    B, H, Sq, Sk = shape
    q, k, v = _attn_inputs(cuda, B, H, Sq, Sk, seed=11, spike=spike)
    outs = {}
    for variant in _variants(0, 1):
        def go():
            o_ref, l_ref = K.attention_fwd(q, k, v, H)
            res = [(o_ref.clone(), l_ref.clone())]
            for _ in range(2):
                o, l = K.attention_fwd(q, k, v, H)
                res.append((o.clone(), l.clone()))
            # graph capture of the same launch, replayed three times
            out = torch.empty_like(o_ref)
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                K.attention_fwd(q, k, v, H, out=out)  # warm-up on the capture stream
            torch.cuda.current_stream().wait_stream(s)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                _, lse_g = K.attention_fwd(q, k, v, H, out=out)
            for _ in range(3):
                out.zero_()
                graph.replay()
                torch.cuda.synchronize()
                res.append((out.clone(), lse_g.clone()))
            return res
        res = _run_variant(K, variant, go)
        o0, l0 = res[0]
        for i, (o, l) in enumerate(res[1:]):
            assert torch.equal(o, o0), f"variant {variant}: output differs on run {i + 1}"
            assert torch.equal(l, l0), f"variant {variant}: LSE differs on run {i + 1}"
        outs[variant] = (o0, l0)
    if 1 in outs:
        assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1]), \
            "lane-local growth test changed the forward's bits"
    # and both are the softmax attention (fp32 reference on a slice of heads)
    qf, kf, vf = (t.float().view(t.shape[0], t.shape[1], H, 64)[:, :, :2].transpose(1, 2) for t in (q, k, v))
    ref = torch.softmax(qf @ kf.transpose(-1, -2) / 8.0, -1) @ vf
    mine = outs[0][0].float().view(B, Sq, H, 64)[:, :, :2].transpose(1, 2)
    assert ((mine - ref).norm() / ref.norm()).item() < 1e-2


@pytest.mark.knob_variants
@pytest.mark.parametrize("shape", [(4, 10, 4096, 4096), (8, 20, 1024, 1024), (3, 10, 1000, 1000), (4, 10, 4096, 77),
                                   (2, 20, 1000, 77)])
@pytest.mark.parametrize("spike", [False, True])
def test_attention_bwd_forms_bit_identical(cuda, shape, spike):
    """The dK/dV / dQ forms give the same bits: the default one-image LDS ring (Q / dO staged once in the transposed-read
    layout), the two-image ring (bwd variant 3) and the 8-wave ping-pong dK/dV (variant 8, and 9 at raised priority;
    self-attention only -- the 77-key cross-attention runs the one-pass attn_bwd_x_kernel under every variant but 7,
    whose dQ + dK/dV launches are checked against the same fp32 reference), each reproducible run to run, on
    ragged (1000-token) and spiked inputs; and the default matches an fp32 autograd reference."""
    from pairwise_sample_optimization_amd import kernels as K
    B, H, Sq, Sk = shape
    q, k, v = _attn_inputs(cuda, B, H, Sq, Sk, seed=17, spike=spike)
    o, lse = K.attention_fwd(q, k, v, H)
    g = torch.Generator(device="cuda").manual_seed(5)
    do = torch.randn(B, Sq, H * 64, device=cuda, generator=g).bfloat16()
    grads = {}
    # 30: two-image ring, 50 / 60: one-image rings of 3 / 4 stages, 80 / 90: 8-wave ping-pong dK/dV (tools build)
    for variant in _variants(0, 30, 50, 60, 80, 90, *([70] if Sk <= 96 else [])):
        def go():
            a = [x.clone() for x in K.attention_bwd(q, k, v, o, lse, do, H)]
            b = K.attention_bwd(q, k, v, o, lse, do, H)
            return a, b
        a, b = _run_variant(K, variant, go)
        for x, y in zip(a, b):
            assert torch.equal(x, y), f"bwd variant {variant}: not reproducible"
        grads[variant] = a
    for variant in [v for v in grads if v and v != 70]:
        for name, x, y in zip(("dq", "dk", "dv"), grads[variant], grads[0]):
            assert torch.equal(x, y), f"bwd variant {variant}: {name} differs from the default form"
    # fp32 reference on two heads
    qf, kf, vf, dof = (t.float().view(B, -1, H, 64)[:, :, :2].transpose(1, 2).detach().requires_grad_(True)
                       for t in (q, k, v, do))
    ref = torch.softmax(qf @ kf.transpose(-1, -2) / 8.0, -1) @ vf
    ref.backward(dof)
    for variant, gv in grads.items():
        if variant not in (0, 70):
            continue
        for name, mine, r in zip(("dq", "dk", "dv"), gv, (qf.grad, kf.grad, vf.grad)):
            m = mine.float().view(B, -1, H, 64)[:, :, :2].transpose(1, 2)
            assert ((m - r).norm() / r.norm()).item() < 2e-2, (variant, name)


@pytest.mark.knob_variants
def test_unet_paired_forward_graph_bit_exact_at_1024(cuda):
    """The paired UNet forward (2 policy + 2 reference images at 1024^2, LoRA on the policy rows) replayed from a
    hipGraph gives the eager forward's bits, for both attention row-max forms."""
    from pairwise_sample_optimization_amd import kernels as K
    from pairwise_sample_optimization_amd.unet import UNet2DConditionModel, UNetConfig
    cfg = UNetConfig.sdxl(128)
    with torch.device(cuda):
        unet = UNet2DConditionModel(cfg)
    unet.init_weights(0)
    unet.add_adapter(SimpleNamespace(r=32, lora_alpha=32))
    unet.lora.init_gaussian(seed=0, b_std=1e-2)
    unet.prepare()
    g = torch.Generator(device="cuda").manual_seed(3)
    n = 2
    x = torch.randn(n, 128, 128, 4, device=cuda, generator=g).bfloat16()
    t = torch.full((n,), 999.0, device=cuda)
    enc = torch.randn(n * 77, 2048, device=cuda, generator=g).bfloat16().view(n, 77, 2048)
    pooled = torch.randn(n, 1280, device=cuda, generator=g).bfloat16()
    tid = torch.tensor([[1024, 1024, 0, 0, 1024, 1024]], device=cuda, dtype=torch.float32).repeat(n, 1)

    def fwd():
        e, _ = unet.forward_nhwc(x, t, enc, pooled, tid, save=False, paired_ref=True)
        return e

    for variant in _variants(0, 1):
        if _lib.KNOBS:
            K.lib().pso_attention_set_variant(variant)
        try:
            with torch.no_grad():
                e0 = fwd().clone()
                e1 = fwd().clone()
                s = torch.cuda.Stream()
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    fwd()
                torch.cuda.current_stream().wait_stream(s)
                graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graph):
                    eg = fwd()
                reps = []
                for _ in range(2):
                    graph.replay()
                    torch.cuda.synchronize()
                    reps.append(eg.clone())
        finally:
            if _lib.KNOBS:
                K.lib().pso_attention_set_variant(0)
        assert torch.equal(e0, e1), f"variant {variant}: eager forward not reproducible"
        for r_ in reps:
            assert torch.equal(r_, e0), f"variant {variant}: graph replay differs from eager"
        assert not torch.equal(e0[:n], e0[n:]), "LoRA must act on the policy half"
        if variant == 0:
            base = e0
        else:
            assert torch.equal(e0, base), "attention variants differ inside the UNet"
    print("paired forward at 1024^2: eager == eager == graph replay, bit for bit (both row-max forms)")


def test_graph_epoch_equals_eager_epoch_fp8(cuda, monkeypatch):
    """train_epoch_graph with the fp8 forward on: after each optimizer step the replayed policy forward must see the
    updated LoRA B stacks (re-quantised inside the captured region).  Epoch losses of the graph run follow the eager
    run's within the eager run-to-run spread; a replay reading the capture-time fp8 copies drifts from it."""
    from pairwise_sample_optimization_amd import kernels as K
    from pairwise_sample_optimization_amd import unet as U
    from pairwise_sample_optimization_amd.trainer import PSOTrainer, compute_time_ids
    from pairwise_sample_optimization_amd.unet import UNet2DConditionModel, UNetConfig
    # lift the occupancy rule (192 tiles) so the sdxl32 products really run on e4m3 and the replay reads the fp8
    # sB cache this test guards
    monkeypatch.setattr(U, "FP8_MIN_TILES", 0)
    monkeypatch.setattr(U, "FP8_ROUND_GAIN", 1e9)  # and the GEGLU round-cost rule: every fp8 kind runs e4m3
    cfg = UNetConfig.sdxl(32)
    P, gas = 1, 2

    def make():
        with torch.device(cuda):
            unet = UNet2DConditionModel(cfg)
        unet.init_weights(0)
        unet.add_adapter(SimpleNamespace(r=16, lora_alpha=16))
        # b_std 3e-3: |Delta| inside the clip range (2e-2 puts every image's log-ratio past log 1.1 at this size, the
        # loss is then exactly log 2 and the LoRA gradient zero -- nothing for the replay to get wrong)
        unet.lora.init_gaussian(seed=1, b_std=3e-3)
        unet.prepare()
        unet.enable_fp8_forward()
        return unet, PSOTrainer(unet, mode="turbo", num_steps=2, gradient_accumulation_steps=gas,
                                train_batch_size=P, lr=2e-4)  # 3e-3 pushes every log-ratio past the clip in 1 step

    (u_e, tr_e), (u_g, tr_g), (u_e2, tr_e2) = make(), make(), make()
    g = torch.Generator(device="cuda").manual_seed(5)
    Bp = P * gas
    enc = torch.randn(Bp, 77, cfg.cross_attention_dim, device=cuda, generator=g).bfloat16()
    pooled = torch.randn(Bp, cfg.text_embed_dim, device=cuda, generator=g).bfloat16()
    tid = compute_time_ids(256, 0, cuda).repeat(Bp, 1)
    buf = tr_e.sample_pairs(enc, pooled, tid, 32, generator=g,
                            reward_fn=lambda x: torch.rand(x.shape[0], device=cuda, generator=g))
    n0 = K.FP8_LAUNCHES[0]
    for epoch in range(4):
        sb = tr_e.shuffle(buf, generator=torch.Generator(device="cuda").manual_seed(100 + epoch))
        tr_e.train_epoch(sb)
        tr_g.train_epoch_graph(sb)
        tr_e2.train_epoch(sb)
    torch.cuda.synchronize()
    assert tr_g._graph is not None
    assert K.FP8_LAUNCHES[0] > n0, "the fp8 forward must run e4m3 GEMMs"
    le, lg, le2 = (torch.stack(t.loss_hist).cpu() for t in (tr_e, tr_g, tr_e2))
    assert (le - 0.6931471805599453).abs().max() > 1e-3, "the LoRA must move the loss (not clipped, not zero)"
    print(f"fp8 graph-vs-eager losses {lg.tolist()} vs {le.tolist()} (eager again {le2.tolist()})")
    assert le[0] / le[1:].min() > 2, "the updates must move the loss"
    # every reduction of the step is ordered (no float atomics): eager == eager == graph replay, bit for bit; a replay
    # of capture-time fp8 copies would miss every update
    assert torch.equal(le, le2) and torch.equal(le, lg), (le, lg, le2)
    assert torch.equal(u_g.lora.master, u_e.lora.master) and torch.equal(u_e.lora.master, u_e2.lora.master)


def test_lora_backward_side_stream_equals_in_line(cuda):
    """with the LoRA weight-gradient closures on the side stream (PSO_SIDE_STREAM=1) the deferred batched
    products are flushed on the compute stream, so every operand they read must be produced there too (v_kv of the
    cross-attention adapters was computed on the side stream).  The gradients must equal the in-line run bit for bit."""
    from pairwise_sample_optimization_amd import kernels as K
    from pairwise_sample_optimization_amd.trainer import PSOTrainer, compute_time_ids
    from pairwise_sample_optimization_amd.unet import UNet2DConditionModel, UNetConfig
    cfg = UNetConfig.sdxl(32)
    with torch.device(cuda):
        unet = UNet2DConditionModel(cfg)
    unet.init_weights(0)
    unet.add_adapter(SimpleNamespace(r=32, lora_alpha=32))
    unet.lora.init_gaussian(seed=1, b_std=3e-3)
    unet.prepare()
    tr = PSOTrainer(unet, mode="turbo", num_steps=2, gradient_accumulation_steps=1, train_batch_size=2)
    tr.auto_step = False
    g = torch.Generator(device="cuda").manual_seed(9)
    enc = torch.randn(2, 77, 2048, device=cuda, generator=g).bfloat16()
    pooled = torch.randn(2, 1280, device=cuda, generator=g).bfloat16()
    tid = compute_time_ids(256, 0, cuda).repeat(2, 1)
    buf = tr.sample_pairs(enc, pooled, tid, 32, generator=g,
                          reward_fn=lambda x: torch.rand(x.shape[0], device=cuda, generator=g))
    sb = tr.shuffle(buf, generator=torch.Generator(device="cuda").manual_seed(1))
    grads = []
    for side in (False, True, False):
        K.SideStream.enabled = side
        try:
            unet.lora.grad.zero_()
            tr.micro_step(tr.micro_batch(sb, 0, 1))
            torch.cuda.synchronize()
            grads.append(unet.lora.grad.clone())
        finally:
            K.SideStream.enabled = False
    assert grads[0].abs().max() > 0
    assert torch.equal(grads[0], grads[2])
    assert torch.equal(grads[0], grads[1])
