"""End-to-end GPU parity of one PSO micro-step (tiny SDXL topology): loss and LoRA gradients of the HIP path vs the
plain-torch fp32 reference of the whole micro-step (oracle UNet + the reference's turbo step / loss formulas)."""
import math
from types import SimpleNamespace

import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref_turbo_lp(sample, eps, prev, sigma, s_up, dt):
    """DP/turbo_inference_with_logprob.py:69-114 in torch (fp32), differentiable in eps."""
    pred = sample - sigma * eps
    deriv = (sample - pred) / sigma
    mean = sample + deriv * dt
    lp = -((prev - mean) ** 2) / (2 * s_up ** 2) - torch.log(s_up) - torch.log(torch.sqrt(2 * torch.as_tensor(math.pi)))
    return lp.mean(dim=tuple(range(1, lp.ndim)))


@pytest.mark.parametrize("P", [1, 2])
def test_micro_step_loss_and_grad_vs_fp32_reference(cuda, P):
    from oracle import sdxl_ref
    from pairwise_sample_optimization_amd import kernels as K
    from pairwise_sample_optimization_amd.trainer import PSOTrainer, compute_time_ids
    from pairwise_sample_optimization_amd.unet import UNet2DConditionModel, UNetConfig
    cfg = UNetConfig.tiny(16)
    with torch.device(cuda):
        unet = UNet2DConditionModel(cfg)
    unet.init_weights(0)
    unet.add_adapter(SimpleNamespace(r=8, lora_alpha=8))
    unet.lora.init_gaussian(seed=1, b_std=0.05)
    tr = PSOTrainer(unet, mode="turbo", num_steps=4, gradient_accumulation_steps=1, train_batch_size=P)
    g = torch.Generator(device="cuda").manual_seed(3)
    enc = torch.randn(P, 77, cfg.cross_attention_dim, device=cuda, generator=g).bfloat16()
    pooled = torch.randn(P, cfg.text_embed_dim, device=cuda, generator=g).bfloat16()
    tid = compute_time_ids(128, 0, cuda).repeat(P, 1)
    buf = tr.sample_pairs(enc, pooled, tid, 16, generator=g,
                          reward_fn=lambda x: torch.rand(x.shape[0], device=cuda, generator=g))
    assert torch.isfinite(buf["lp"]).all() and torch.isfinite(buf["x_final"]).all()
    sb = tr.shuffle(buf, generator=g)
    mb = tr.micro_batch(sb, 0)
    st = unet.lora
    st.grad.zero_()
    tr.auto_step = False  # no optimizer step inside: inspect the accumulated grads
    loss = tr.micro_step(mb)
    mine_loss = loss.item()
    mine_grads = {k: v.clone() for k, v in st.grad_dict_peft().items()}
    # ---- fp32 reference of the same micro-step ----
    sd = sdxl_ref.sd_to(unet.state_dict(), cuda)
    leaf = {k: v.float().clone().requires_grad_(True) for k, v in st.state_dict_peft().items()}
    ocfg = dict(time_proj_dim=cfg.time_proj_dim, addition_time_embed_dim=cfg.addition_time_embed_dim)
    x_in = K.nhwc_to_nchw(mb.unet_in).float()
    ep = sdxl_ref.unet_forward(sd, x_in, mb.t, mb.enc.float(), mb.pooled.float(), mb.tid, lora=leaf, cfg=ocfg)
    with torch.no_grad():
        er = sdxl_ref.unet_forward(sd, x_in, mb.t, mb.enc.float(), mb.pooled.float(), mb.tid, lora=None, cfg=ocfg)
    # the reference casts UNet outputs to fp32 after a bf16 autocast forward: round eps to bf16 values
    ep = ep + (ep.bfloat16().float() - ep).detach()
    er = er.bfloat16().float()
    xs = mb.x.permute(0, 3, 1, 2)
    xp = mb.x_next.permute(0, 3, 1, 2)
    c = mb.coef
    sig, su, dt = (c[:, i].view(-1, 1, 1, 1) for i in (0, 1, 2))
    lp_p = _ref_turbo_lp(xs, ep, xp, sig, su, dt)
    lp_r = _ref_turbo_lp(xs, er, xp, sig, su, dt)
    pref = K.preference(mb.rewards, 0)
    d = (lp_p - lp_r).view(P, 2)
    ratio = torch.clamp(torch.exp(d), 0.9, 1.1)
    ref_loss = -torch.log(torch.sigmoid(50 * torch.log(ratio[:, 0]) * pref[:, 0] +
                                        50 * torch.log(ratio[:, 1]) * pref[:, 1])).mean()
    (ref_loss / tr.gas_total).backward()  # accelerator.backward divides by gradient_accumulation_steps = gas*T
    # the reference's own numerics: the UNet cast to weight_dtype = bf16 (T:299-321) run under accelerate's bf16
    # autocast -- bf16 hidden states and residual stream, fp32 norms / softmax
    sd16 = sdxl_ref.sd_to(unet.state_dict(), cuda, torch.bfloat16)
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        ep16 = sdxl_ref.unet_forward(sd16, x_in, mb.t, mb.enc.float(), mb.pooled.float(), mb.tid,
                                     lora={k: v.detach() for k, v in leaf.items()}, cfg=ocfg).float()
        er16 = sdxl_ref.unet_forward(sd16, x_in, mb.t, mb.enc.float(), mb.pooled.float(), mb.tid, lora=None,
                                     cfg=ocfg).float()
    with torch.no_grad():
        d16 = (_ref_turbo_lp(xs, ep16, xp, sig, su, dt) - _ref_turbo_lp(xs, er16, xp, sig, su, dt)).view(P, 2)
        r16 = torch.clamp(torch.exp(d16), 0.9, 1.1)
        loss16 = -torch.log(torch.sigmoid(50 * torch.log(r16[:, 0]) * pref[:, 0] +
                                          50 * torch.log(r16[:, 1]) * pref[:, 1])).mean().item()
    rel = abs(mine_loss - ref_loss.item()) / abs(ref_loss.item())
    num = sum(((mine_grads[k] - v.grad) ** 2).sum().item() for k, v in leaf.items())
    den = sum((v.grad ** 2).sum().item() for v in leaf.values())
    grel = (num / max(den, 1e-30)) ** 0.5
    rel16 = abs(loss16 - ref_loss.item()) / abs(ref_loss.item())
    print(f"P={P}: loss mine={mine_loss:.6f} fp32-ref={ref_loss.item():.6f} torch-bf16={loss16:.6f} "
          f"rel(mine)={rel:.2e} rel(torch-bf16)={rel16:.2e}; grad rel={grel:.3e}")
    # Both bf16 paths see eps_pol - eps_ref (the LoRA effect) through ~1% bf16 activation noise, which beta=50
    # amplifies into the loss.  At this tiny topology (64-128 channels, b_std 0.05) the HIP path measured 4.4e-3 /
    # 7.9e-3 against torch-bf16's 1.8e-3 / 3.7e-3, so the bar here is 3x the torch-bf16 distance + 2e-3; the strict
    # 1.5x form is applied at the bench configurations' full size (tests/test_gpu_fullsize.py, where the HIP path
    # lands closer to fp32 than torch-bf16).  The loss kernel alone on identical eps: 5e-5 (test_gpu_pso_loss).
    assert rel <= 3.0 * rel16 + 2e-3
    if den > 0:
        assert grel < 1e-1


def test_optimizer_step_matches_torch_adamw(cuda):
    from pairwise_sample_optimization_amd import kernels as K
    n = 10_000
    g = torch.Generator(device="cuda").manual_seed(0)
    p = torch.randn(n, device=cuda, generator=g)
    grad = torch.randn(n, device=cuda, generator=g) * 3
    p_ref = p.clone().requires_grad_(True)
    opt = torch.optim.AdamW([p_ref], lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2)
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    for step in range(1, 4):
        gg = grad * step
        p_ref.grad = gg.clone()
        torch.nn.utils.clip_grad_norm_([p_ref], 1.0)
        opt.step()
        clip = K.grad_clip_coef(gg, 1.0)
        K.adamw_step(p, gg, m, v, 1e-3, (0.9, 0.999), 1e-8, 1e-2, step, clip=clip)
    assert (p - p_ref.detach()).abs().max().item() < 1e-5


def test_checkpoint_save_load_roundtrip(cuda, tmp_path):
    """save_state -> fresh trainer -> load_state restores LoRA weights, AdamW moments and counters (T:886-890)."""
    from pairwise_sample_optimization_amd import lora_io
    from pairwise_sample_optimization_amd.trainer import PSOTrainer
    from pairwise_sample_optimization_amd.unet import UNet2DConditionModel, UNetConfig
    mk = lambda: UNet2DConditionModel(UNetConfig.tiny(16))
    with torch.device(cuda):
        u1, u2 = mk(), mk()
    u1.init_weights(0)
    u2.init_weights(0)
    u1.add_adapter(SimpleNamespace(r=8, lora_alpha=8))
    u2.add_adapter(SimpleNamespace(r=8, lora_alpha=8, seed=5))
    u1.lora.init_gaussian(1, b_std=1e-2)
    t1 = PSOTrainer(u1, mode="turbo", num_steps=4)
    t2 = PSOTrainer(u2, mode="turbo", num_steps=4)
    t1.exp_avg.normal_()
    t1.exp_avg_sq.uniform_()
    t1.opt_step, t1.n_micro = 7, 21
    lora_io.save_state(t1, str(tmp_path))
    lora_io.load_state(t2, str(tmp_path))
    assert torch.equal(u1.lora.master, u2.lora.master)
    assert torch.equal(t1.exp_avg, t2.exp_avg) and torch.equal(t1.exp_avg_sq, t2.exp_avg_sq)
    assert (t2.opt_step, t2.n_micro) == (7, 21)
    x = torch.randn(2, 4, 16, 16, device=cuda)
    enc = torch.randn(2, 77, 128, device=cuda)
    cond = {"text_embeds": torch.randn(2, 64, device=cuda),
            "time_ids": torch.tensor([[128.0, 128, 0, 0, 128, 128]] * 2, device=cuda)}
    with torch.no_grad():
        e1 = u1(x, 999.0, enc, added_cond_kwargs=cond).sample
        e2 = u2(x, 999.0, enc, added_cond_kwargs=cond).sample
    assert torch.equal(e1, e2)


@pytest.mark.parametrize("mode", ["turbo", "dmd"])
def test_batched_window_equals_sequential_micro_steps(cuda, mode):
    """One batched pass over a whole accumulation window == the reference's sequential micro-steps
    (T:755-861): same summed LoRA gradient (up to fp32 summation order and bf16 tile effects), same mean loss."""
    from pairwise_sample_optimization_amd.trainer import PSOTrainer, compute_time_ids
    from pairwise_sample_optimization_amd.unet import UNet2DConditionModel, UNetConfig
    cfg = UNetConfig.tiny(16)
    with torch.device(cuda):
        unet = UNet2DConditionModel(cfg)
    unet.init_weights(0)
    unet.add_adapter(SimpleNamespace(r=8, lora_alpha=8))
    unet.lora.init_gaussian(seed=1, b_std=0.05)
    P, gas, N = 2, 2, 3
    tr = PSOTrainer(unet, mode=mode, num_steps=N, gradient_accumulation_steps=gas, train_batch_size=P,
                    num_reward=2)
    tr.auto_step = False
    g = torch.Generator(device="cuda").manual_seed(5)
    Bp = P * gas
    enc = torch.randn(Bp, 77, cfg.cross_attention_dim, device=cuda, generator=g).bfloat16()
    pooled = torch.randn(Bp, cfg.text_embed_dim, device=cuda, generator=g).bfloat16()
    tid = compute_time_ids(128, 0, cuda).repeat(Bp, 1)
    buf = tr.sample_pairs(enc, pooled, tid, 16, generator=g,
                          reward_fn=lambda x: torch.rand(x.shape[0], 2, device=cuda, generator=g))
    sb = tr.shuffle(buf, generator=g)
    assert sb.n_micro == gas * (N - 1) == tr.gas_total
    st = unet.lora
    st.grad.zero_()
    g1 = torch.Generator(device="cuda").manual_seed(9)
    seq = [tr.micro_step(tr.micro_batch(sb, s), generator=g1) for s in range(sb.n_micro)]
    seq_grad = st.grad.clone()
    seq_loss = torch.stack(seq).mean().item()
    st.grad.zero_()
    tr.n_micro = 0
    g1 = torch.Generator(device="cuda").manual_seed(9)
    # the reward column draws (turbo, T:405) come from one generator call instead of gas*T: draw them the same way
    if mode == "turbo":
        idx = torch.cat([torch.randint(0, 2, (P,), device=cuda, generator=g1) for _ in range(sb.n_micro)])
        g1 = None
        saved = torch.randint
        torch.randint = lambda *a, **k: idx
    try:
        loss = tr.micro_step(tr.micro_batch(sb, 0, sb.n_micro), generator=g1)
    finally:
        if mode == "turbo":
            torch.randint = saved
    rel = ((st.grad - seq_grad).norm() / seq_grad.norm()).item()
    print(f"{mode}: batched-vs-sequential grad rel {rel:.2e}, loss {loss.item():.6f} vs {seq_loss:.6f}")
    assert seq_grad.norm() > 0
    # each path carries its own bf16 rounding (different M -> different tile shapes / split reductions), ~2-3 % rel-L2
    # vs fp32 apiece (test_micro_step_loss_and_grad_vs_fp32_reference); their difference is bounded by the sum
    assert rel < 4e-2
    # beta = 50 multiplies the bf16 eps rounding of the log-ratios: measured up to 4.1e-3 rel (turbo; 2.5e-3 DMD2)
    # across boxes and attention row-sum forms, so the bar is 8e-3 (a wrong gradient/loss path is off by O(1))
    assert abs(loss.item() - seq_loss) < 8e-3 * abs(seq_loss) + 1e-6
    with pytest.raises(ValueError):
        tr.n_micro = 1
        tr.micro_step(tr.micro_batch(sb, 0, sb.n_micro))


def test_graph_epoch_equals_eager_epoch(cuda):
    """train_epoch_graph (the epoch captured once as a hipGraph, then replayed with fresh shuffled inputs) leaves the
    same LoRA parameters, AdamW moments and losses as the eager train_epoch over the same shuffles -- bit for bit, and
    two eager runs agree bit for bit too: the forward has no float atomics and every LoRA weight-gradient product is
    reduced in a fixed order (pso_gemm_tn_rank_batch_ws / pso_gemm_tn_ws), as the reference's cuBLAS dW GEMMs are
    (T:857).  Ranks 8 (64 x 64 TN slices) and 32 (the batched rank kernel) cover both reduction paths."""
    from pairwise_sample_optimization_amd.trainer import PSOTrainer, compute_time_ids
    from pairwise_sample_optimization_amd.unet import UNet2DConditionModel, UNetConfig
    cfg = UNetConfig.tiny(16)
    P, gas = 2, 2

    for r in (8, 32):
        def make():
            with torch.device(cuda):
                unet = UNet2DConditionModel(cfg)
            unet.init_weights(0)
            unet.add_adapter(SimpleNamespace(r=r, lora_alpha=r))
            unet.lora.init_gaussian(seed=1, b_std=0.05)
            unet.prepare()
            return unet, PSOTrainer(unet, mode="turbo", num_steps=2, gradient_accumulation_steps=gas,
                                    train_batch_size=P, lr=1e-3)

        u_e, tr_e = make()
        u_g, tr_g = make()
        u_e2, tr_e2 = make()  # a second eager run: must agree with the first bit for bit
        g = torch.Generator(device="cuda").manual_seed(5)
        Bp = P * gas
        enc = torch.randn(Bp, 77, cfg.cross_attention_dim, device=cuda, generator=g).bfloat16()
        pooled = torch.randn(Bp, cfg.text_embed_dim, device=cuda, generator=g).bfloat16()
        tid = compute_time_ids(128, 0, cuda).repeat(Bp, 1)
        buf = tr_e.sample_pairs(enc, pooled, tid, 16, generator=g,
                                reward_fn=lambda x: torch.rand(x.shape[0], device=cuda, generator=g))
        for epoch in range(3):  # capture on the first call, replay on the next two (different shuffles)
            sb = tr_e.shuffle(buf, generator=torch.Generator(device="cuda").manual_seed(100 + epoch))
            tr_e.train_epoch(sb)
            tr_g.train_epoch_graph(sb)
            tr_e2.train_epoch(sb)
        torch.cuda.synchronize()
        assert tr_g._graph is not None and tr_g.opt_step == tr_e.opt_step == 3
        le = torch.stack(tr_e.loss_hist).cpu()
        lg = torch.stack(tr_g.loss_hist).cpu()
        le2 = torch.stack(tr_e2.loss_hist).cpu()
        print(f"r={r}: graph losses {lg.tolist()} eager {le.tolist()} eager again {le2.tolist()}")
        assert le[-1] < 0.5 * le[0]  # the epochs train (a replay on stale weights or inputs would not match below)
        assert torch.equal(le, le2), (le, le2)
        assert torch.equal(le, lg), (le, lg)
        assert torch.equal(u_e.lora.master, u_e2.lora.master)
        assert torch.equal(u_e.lora.master, u_g.lora.master)
        for a, b in ((tr_e.exp_avg, tr_g.exp_avg), (tr_e.exp_avg_sq, tr_g.exp_avg_sq)):
            assert torch.equal(a, b)


def test_full_unet_micro_step_vs_fp32_reference(cuda):
    """Full-UNet training (BASELINE C3 / C4): one PSO micro-step with every UNet parameter trainable and a frozen
    reference UNet -- loss and the gradients of all parameters vs the plain-torch fp32 reference of the micro-step."""
    from oracle import sdxl_ref
    from pairwise_sample_optimization_amd import kernels as K
    from pairwise_sample_optimization_amd.trainer import PSOTrainer, compute_time_ids
    from pairwise_sample_optimization_amd.unet import UNet2DConditionModel, UNetConfig
    cfg = UNetConfig.tiny(16)
    P = 1

    def make():
        with torch.device(cuda):
            u = UNet2DConditionModel(cfg)
        u.init_weights(0)
        return u

    unet, ref_unet = make(), make()
    fg = unet.enable_full_grads()
    ref_unet.prepare()
    tr = PSOTrainer(unet, mode="turbo", num_steps=4, gradient_accumulation_steps=1, train_batch_size=P,
                    ref_unet=ref_unet)
    g = torch.Generator(device="cuda").manual_seed(3)
    enc = torch.randn(P, 77, cfg.cross_attention_dim, device=cuda, generator=g).bfloat16()
    pooled = torch.randn(P, cfg.text_embed_dim, device=cuda, generator=g).bfloat16()
    tid = compute_time_ids(128, 0, cuda).repeat(P, 1)
    buf = tr.sample_pairs(enc, pooled, tid, 16, generator=g,
                          reward_fn=lambda x: torch.rand(x.shape[0], device=cuda, generator=g))
    sb = tr.shuffle(buf, generator=g)
    mb = tr.micro_batch(sb, 0)
    fg.grad.zero_()
    tr.auto_step = False
    mine_loss = tr.micro_step(mb).item()
    mine = {unet._unmap_key(n): fg.g(p).clone() for n, p in unet.named_parameters()}
    # the reference pass on its own stream (default) and in line: the same loss bits, the same gradients (up to the
    # f32-atomic order of the full-UNet bias / norm parameter sums)
    from pairwise_sample_optimization_amd import trainer as T_
    assert T_._REF_STREAM
    T_._REF_STREAM = False
    try:
        g0 = fg.grad.clone()
        fg.grad.zero_()
        inline_loss = tr.micro_step(mb).item()
        assert inline_loss == mine_loss
        assert ((fg.grad - g0).norm() / g0.norm()).item() < 1e-5
    finally:
        T_._REF_STREAM = True
    sd = sdxl_ref.sd_to(unet.state_dict(), cuda)
    leaf = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
    ocfg = dict(time_proj_dim=cfg.time_proj_dim, addition_time_embed_dim=cfg.addition_time_embed_dim)
    x_in = K.nhwc_to_nchw(mb.unet_in).float()
    ep = sdxl_ref.unet_forward(leaf, x_in, mb.t, mb.enc.float(), mb.pooled.float(), mb.tid, lora=None, cfg=ocfg)
    with torch.no_grad():
        er = sdxl_ref.unet_forward(sd, x_in, mb.t, mb.enc.float(), mb.pooled.float(), mb.tid, lora=None, cfg=ocfg)
    ep = ep + (ep.bfloat16().float() - ep).detach()
    er = er.bfloat16().float()
    xs, xp, c = mb.x.permute(0, 3, 1, 2), mb.x_next.permute(0, 3, 1, 2), mb.coef
    sig, su, dt = (c[:, i].view(-1, 1, 1, 1) for i in (0, 1, 2))
    pref = K.preference(mb.rewards, 0)
    d = (_ref_turbo_lp(xs, ep, xp, sig, su, dt) - _ref_turbo_lp(xs, er, xp, sig, su, dt)).view(P, 2)
    ratio = torch.clamp(torch.exp(d), 0.9, 1.1)
    ref_loss = -torch.log(torch.sigmoid(50 * torch.log(ratio[:, 0]) * pref[:, 0] +
                                        50 * torch.log(ratio[:, 1]) * pref[:, 1])).mean()
    (ref_loss / tr.gas_total).backward()
    num = sum(((mine[k] - v.grad) ** 2).sum().item() for k, v in leaf.items())
    den = sum((v.grad ** 2).sum().item() for v in leaf.values())
    grel = (num / den) ** 0.5
    rel = abs(mine_loss - ref_loss.item()) / abs(ref_loss.item())
    print(f"full-UNet micro-step: loss mine={mine_loss:.6f} fp32={ref_loss.item():.6f} rel={rel:.2e}; "
          f"grad rel over {len(leaf)} tensors={grel:.3e}")
    assert rel < 2e-2
    assert grel < 1e-1


def test_dmd_sampling_noise_per_pair_member(cuda, monkeypatch):
    """DMD2 re-noising: each trajectory of a pair is its own pipeline call (D:585-618) whose step draws ONE (1,C,H,W)
    noise shared by that call's batch (DP/distilled_inference_with_logprob.py:123-126) -- so the two members of a
    pair get different draws while images with the same member index share one."""
    from pairwise_sample_optimization_amd import trainer as T_
    from pairwise_sample_optimization_amd.trainer import PSOTrainer, compute_time_ids
    from pairwise_sample_optimization_amd.unet import UNet2DConditionModel, UNetConfig
    cfg = UNetConfig.tiny(16)
    with torch.device(cuda):
        unet = UNet2DConditionModel(cfg)
    unet.init_weights(0)
    unet.add_adapter(SimpleNamespace(r=8, lora_alpha=8))
    tr = PSOTrainer(unet, mode="dmd", num_steps=3, train_batch_size=1)
    seen = []
    real = T_.K.step_logprob

    def spy(mode, x, eps, coef, prev=None, noise=None, noise_shared=False):
        if noise is not None and noise.abs().sum() > 0:
            seen.append((noise.clone(), noise_shared))
        return real(mode, x, eps, coef, prev=prev, noise=noise, noise_shared=noise_shared)

    monkeypatch.setattr(T_.K, "step_logprob", spy)
    B = 3
    g = torch.Generator(device="cuda").manual_seed(4)
    enc = torch.randn(B, 77, cfg.cross_attention_dim, device=cuda, generator=g).bfloat16()
    pooled = torch.randn(B, cfg.text_embed_dim, device=cuda, generator=g).bfloat16()
    tr.sample_pairs(enc, pooled, compute_time_ids(128, 0, cuda).repeat(B, 1), 16, generator=g)
    assert len(seen) == 2  # N - 1 stochastic transitions
    for noise, shared in seen:
        n = noise if not shared else noise.expand(2 * B, *noise.shape[1:])
        assert not torch.equal(n[0], n[1])                       # the two members of a pair differ
        for b in range(1, B):
            assert torch.equal(n[2 * b], n[0]) and torch.equal(n[2 * b + 1], n[1])  # shared across prompts


def test_graph_epoch_falls_back_to_eager_for_full_unet(cuda):
    """train_epoch_graph must not capture a full-UNet epoch: its optimizer step rebuilds the kernel-layout weight
    caches as new tensors that a replayed graph would not see.  Two epochs run eagerly and train."""
    from pairwise_sample_optimization_amd.trainer import PSOTrainer, compute_time_ids
    from pairwise_sample_optimization_amd.unet import UNet2DConditionModel, UNetConfig
    cfg = UNetConfig.tiny(16)

    def make():
        with torch.device(cuda):
            u = UNet2DConditionModel(cfg)
        u.init_weights(0)
        return u

    unet, ref = make(), make()
    unet.enable_full_grads()
    ref.prepare()
    tr = PSOTrainer(unet, mode="turbo", num_steps=2, train_batch_size=1, ref_unet=ref, lr=1e-4)
    g = torch.Generator(device="cuda").manual_seed(6)
    enc = torch.randn(1, 77, cfg.cross_attention_dim, device=cuda, generator=g).bfloat16()
    pooled = torch.randn(1, cfg.text_embed_dim, device=cuda, generator=g).bfloat16()
    buf = tr.sample_pairs(enc, pooled, compute_time_ids(128, 0, cuda), 16, generator=g,
                          reward_fn=lambda x: torch.rand(x.shape[0], device=cuda, generator=g))
    w0 = unet.conv_out.weight.detach().clone()
    for _ in range(2):
        tr.train_epoch_graph(tr.shuffle(buf, generator=g))
    torch.cuda.synchronize()
    assert getattr(tr, "_graph", None) is None and tr.opt_step == 2
    assert torch.isfinite(torch.stack(tr.loss_hist)).all()
    assert not torch.equal(unet.conv_out.weight, w0)


def test_use_8bit_adam_trains_and_checkpoints(cuda, tmp_path):
    """train.use_8bit_adam (the reference default, config_sdxl_turbo_dpo.py:86, T:427-435): PSOTrainer.from_config
    selects the blockwise 8-bit AdamW; three epochs move the LoRA weights the way fp32 AdamW does (same direction,
    magnitudes within the 8-bit state's rounding), and save_state / load_state round-trip its codes and scales."""
    from pairwise_sample_optimization_amd import lora_io
    from pairwise_sample_optimization_amd.config import config_sdxl_turbo_dpo
    from pairwise_sample_optimization_amd.trainer import PSOTrainer, compute_time_ids
    from pairwise_sample_optimization_amd.unet import UNet2DConditionModel, UNetConfig
    cfg = UNetConfig.tiny(16)
    c = config_sdxl_turbo_dpo.get_config()
    c.sample.num_steps, c.train.distilled_train_steps = 2, 1
    c.train.batch_size, c.train.gradient_accumulation_steps, c.train.learning_rate = 2, 1, 1e-3

    def make(adam8):
        with torch.device(cuda):
            u = UNet2DConditionModel(cfg)
        u.init_weights(0)
        u.add_adapter(SimpleNamespace(r=8, lora_alpha=8))
        u.lora.init_gaussian(seed=1, b_std=2e-3)
        u.prepare()
        c.train.use_8bit_adam = adam8
        return u, PSOTrainer.from_config(u, c, mode="turbo")

    (u8, t8), (u32, t32) = make(True), make(False)
    assert t8.adam8 is not None and t8.exp_avg is None and t32.adam8 is None
    m0 = u8.lora.master.clone()
    g = torch.Generator(device="cuda").manual_seed(5)
    enc = torch.randn(2, 77, cfg.cross_attention_dim, device=cuda, generator=g).bfloat16()
    pooled = torch.randn(2, cfg.text_embed_dim, device=cuda, generator=g).bfloat16()
    tid = compute_time_ids(128, 0, cuda).repeat(2, 1)
    buf = t8.sample_pairs(enc, pooled, tid, 16, generator=g,
                          reward_fn=lambda x: torch.rand(x.shape[0], device=cuda, generator=g))
    for epoch in range(3):
        for t in (t8, t32):
            t.train_epoch(t.shuffle(buf, generator=torch.Generator(device="cuda").manual_seed(100 + epoch)))
    torch.cuda.synchronize()
    d8, d32 = u8.lora.master - m0, u32.lora.master - m0
    assert t8.opt_step == 3 and d8.abs().max() > 0
    # the 8-bit step zeroed the gradient it read (pads included: no kernel writes them)
    assert u8.lora.grad.abs().max().item() == 0 and u32.lora.grad.abs().max().item() == 0
    cos = (d8 * d32).sum() / (d8.norm() * d32.norm())
    print(f"8-bit vs fp32 AdamW update: cos {cos.item():.4f}, norm ratio {(d8.norm() / d32.norm()).item():.4f}")
    assert cos > 0.95 and 0.8 < (d8.norm() / d32.norm()).item() < 1.25
    lora_io.save_state(t8, str(tmp_path))
    u2, t2 = make(True)
    lora_io.load_state(t2, str(tmp_path))
    for a, b in ((t8.adam8.qm, t2.adam8.qm), (t8.adam8.qv, t2.adam8.qv), (t8.adam8.am, t2.adam8.am),
                 (t8.adam8.av, t2.adam8.av), (u8.lora.master, u2.lora.master)):
        assert torch.equal(a, b)
    assert t2.opt_step == 3
