"""End-to-end GPU parity of one DreamBooth PSO micro-step (config 5, DB:1720-1964; tiny SDXL topology): loss and LoRA
gradients of the HIP path (VAE encoder + UNet fwd/bwd + fused loss) vs the plain-torch fp32 reference of the same
micro-step on the same latents / noise / timesteps (oracle UNet + the restated loss).  The DreamBooth trainer itself
cannot be imported here, so the loss half is pinned to the restatement only (parity unpinned)."""
from types import SimpleNamespace

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("loss_type,B", [("pso_db", 1), ("pso", 2)])
def test_dreambooth_micro_step_vs_fp32_reference(cuda, loss_type, B):
    from oracle import sdxl_ref
    from pairwise_sample_optimization_amd import kernels as K
    from pairwise_sample_optimization_amd.dreambooth import DreamBoothPSOTrainer
    from pairwise_sample_optimization_amd.trainer import compute_time_ids
    from pairwise_sample_optimization_amd.unet import UNet2DConditionModel, UNetConfig
    from pairwise_sample_optimization_amd.vae import AutoencoderKL, VAEConfig
    cfg = UNetConfig.tiny(16)
    with torch.device(cuda):
        unet = UNet2DConditionModel(cfg)
        vae = AutoencoderKL(VAEConfig.tiny())
    unet.init_weights(0)
    vae.init_weights(2)
    unet.add_adapter(SimpleNamespace(r=8, lora_alpha=8))
    unet.lora.init_gaussian(seed=1, b_std=0.05)
    beta = 5.0 if loss_type == "pso_db" else 20.0
    tr = DreamBoothPSOTrainer(unet, vae, loss_type=loss_type, beta_pso=beta, gradient_accumulation_steps=1)
    tr.auto_step = False
    g = torch.Generator(device="cuda").manual_seed(4)
    pix = torch.rand(2 * B, 3, 128, 128, device=cuda, generator=g) * 2 - 1
    enc = torch.randn(B, 77, cfg.cross_attention_dim, device=cuda, generator=g).bfloat16()
    pooled = torch.randn(B, cfg.text_embed_dim, device=cuda, generator=g).bfloat16()
    tid = compute_time_ids(128, 0, cuda).repeat(B, 1)
    st = unet.lora
    st.grad.zero_()
    gi = torch.Generator(device="cuda").manual_seed(11)
    loss = tr.micro_step(pix, enc, pooled, tid, generator=gi).item()
    mine = {k: v.clone() for k, v in st.grad_dict_peft().items()}
    # the same inputs again (same generator seed), then the fp32 reference micro-step
    gi = torch.Generator(device="cuda").manual_seed(11)
    inp = tr.prepare_inputs(pix, gi)
    sd = sdxl_ref.sd_to(unet.state_dict(), cuda)
    leaf = {k: v.float().clone().requires_grad_(True) for k, v in st.state_dict_peft().items()}
    ocfg = dict(time_proj_dim=cfg.time_proj_dim, addition_time_embed_dim=cfg.addition_time_embed_dim)
    x_in = K.nhwc_to_nchw(inp["unet_in"]).float()
    e2, p2, t2 = enc.float().repeat(2, 1, 1), pooled.float().repeat(2, 1), tid.repeat(2, 1)
    ep = sdxl_ref.unet_forward(sd, x_in, inp["t"], e2, p2, t2, lora=leaf, cfg=ocfg)
    ep = ep + (ep.bfloat16().float() - ep).detach()  # bf16-autocast output values, fp32 gradient path
    s = inp["sigma"].view(-1, 1, 1, 1)
    nz, x0 = inp["noisy"].permute(0, 3, 1, 2), inp["x0"].permute(0, 3, 1, 2)
    per = lambda e: ((s ** -2.0) * ((e * (-s) + nz) - x0) ** 2).reshape(2 * B, -1).mean(1)
    lw, ll = per(ep).chunk(2)
    md = lw - 0.1 * ll
    if loss_type == "pso":
        with torch.no_grad():
            er = sdxl_ref.unet_forward(sd, x_in, inp["t"], e2, p2, t2, lora=None, cfg=ocfg).bfloat16().float()
        rw, rl = per(er).chunk(2)
        ref = -torch.nn.functional.logsigmoid(beta * ((rw - 0.1 * rl) - md)).mean()
    else:
        ref = torch.relu(1 - beta * (-md)).mean()
    ref = ref + 0.5 * ll.mean()
    ref.backward()
    rel = abs(loss - ref.item()) / abs(ref.item())
    num = sum(((mine[k] - v.grad) ** 2).sum().item() for k, v in leaf.items())
    den = sum((v.grad ** 2).sum().item() for v in leaf.values())
    grel = (num / max(den, 1e-30)) ** 0.5
    print(f"{loss_type} B={B}: loss mine={loss:.6f} fp32-ref={ref.item():.6f} rel={rel:.2e} grad rel={grel:.3e}")
    assert rel < 2e-2
    assert den > 0 and grel < 1e-1


@pytest.mark.timeout(900)
def test_dreambooth_micro_step_fp8_at_1024(cuda):
    """BASELINE config 5 at its per-GPU workload: the DreamBooth PSO micro-step (DB:1720-1964, recipe
    scripts/pso_dog.sh: pso_db, beta 5, rank 16, 1 instance + 1 negative image) at 1024^2 with the full SDXL UNet and
    VAE encoder, with the fp8 forward on (enable_fp8_forward: e4m3 cross q and GEGLU proj; bf16 backward), against
    the fp32 oracle micro-step on the same latents / noise / timesteps.  The bf16 forward runs beside it on the same
    inputs so the fp8 cost is visible.  Stated fp8 tolerance: loss rel <= 5e-3, LoRA grad rel <= 5e-2 (e4m3 has 3
    mantissa bits; the bf16 forward's bars are 2e-2 / 1e-1; round 3 also ran the self-attention q/k/v in e4m3: grad
    rel 8.6e-2, 7.5e-2 of it from q/k/v alone, tools/diag_fp8_grads.py)."""
    from oracle import sdxl_ref
    from pairwise_sample_optimization_amd import kernels as K
    from pairwise_sample_optimization_amd.dreambooth import DreamBoothPSOTrainer
    from pairwise_sample_optimization_amd.trainer import compute_time_ids
    from pairwise_sample_optimization_amd.unet import UNet2DConditionModel, UNetConfig
    from pairwise_sample_optimization_amd.vae import AutoencoderKL, VAEConfig
    cfg = UNetConfig.sdxl(128)
    B, beta = 1, 5.0
    with torch.device(cuda):
        unet = UNet2DConditionModel(cfg)
        vae = AutoencoderKL(VAEConfig())
    unet.init_weights(0)
    vae.init_weights(2)
    unet.add_adapter(SimpleNamespace(r=16, lora_alpha=16))
    unet.lora.init_gaussian(seed=1, b_std=5e-3)
    unet.prepare()
    tr = DreamBoothPSOTrainer(unet, vae, loss_type="pso_db", beta_pso=beta, gradient_accumulation_steps=1)
    tr.auto_step = False
    g = torch.Generator(device="cuda").manual_seed(4)
    pix = torch.rand(2 * B, 3, 1024, 1024, device=cuda, generator=g) * 2 - 1
    enc = torch.randn(B, 77, 2048, device=cuda, generator=g).bfloat16()
    pooled = torch.randn(B, 1280, device=cuda, generator=g).bfloat16()
    tid = compute_time_ids(1024, 0, cuda).repeat(B, 1)
    st = unet.lora
    res = {}
    for fp8 in (False, True):
        unet.enable_fp8_forward(fp8)
        st.grad.zero_()
        loss = tr.micro_step(pix, enc, pooled, tid, generator=torch.Generator(device="cuda").manual_seed(11)).item()
        res[fp8] = (loss, {k: v.clone() for k, v in st.grad_dict_peft().items()})
    unet.enable_fp8_forward(False)
    inp = tr.prepare_inputs(pix, torch.Generator(device="cuda").manual_seed(11))
    sd = sdxl_ref.sd_to(unet.state_dict(), cuda)
    leaf = {k: v.float().clone().requires_grad_(True) for k, v in st.state_dict_peft().items()}
    ocfg = dict(time_proj_dim=cfg.time_proj_dim, addition_time_embed_dim=cfg.addition_time_embed_dim)
    x_in = K.nhwc_to_nchw(inp["unet_in"]).float()
    e2, p2, t2 = enc.float().repeat(2, 1, 1), pooled.float().repeat(2, 1), tid.repeat(2, 1)
    s = inp["sigma"].view(-1, 1, 1, 1)
    nz, x0 = inp["noisy"].permute(0, 3, 1, 2), inp["x0"].permute(0, 3, 1, 2)
    per = lambda e: ((s ** -2.0) * ((e * (-s) + nz) - x0) ** 2).reshape(2 * B, -1).mean(1)
    # image by image (one fp32 1024^2 graph at a time); the loss couples them only through lw / ll
    outs = [sdxl_ref.unet_forward(sd, x_in[i:i + 1], inp["t"][i:i + 1], e2[i:i + 1], p2[i:i + 1], t2[i:i + 1],
                                  lora={k: v.detach() for k, v in leaf.items()}, cfg=ocfg).detach()
            for i in range(2 * B)]
    ep = torch.cat(outs).bfloat16().float().requires_grad_(True)
    lw, ll = per(ep).chunk(2)
    ref = torch.relu(1 - beta * (-(lw - 0.1 * ll))).mean() + 0.5 * ll.mean()
    ref.backward()
    for i in range(2 * B):
        out = sdxl_ref.unet_forward(sd, x_in[i:i + 1], inp["t"][i:i + 1], e2[i:i + 1], p2[i:i + 1], t2[i:i + 1],
                                    lora=leaf, cfg=ocfg)
        (out * ep.grad[i:i + 1]).sum().backward()
        del out
    den = sum((v.grad ** 2).sum().item() for v in leaf.values())
    rel, grel = {}, {}
    for fp8, (loss, mine) in res.items():
        rel[fp8] = abs(loss - ref.item()) / abs(ref.item())
        grel[fp8] = (sum(((mine[k] - v.grad) ** 2).sum().item() for k, v in leaf.items()) / max(den, 1e-30)) ** 0.5
    print(f"C5 DreamBooth @1024 (pso_db, r=16): loss fp32 {ref.item():.6f} bf16 {res[False][0]:.6f} "
          f"fp8 {res[True][0]:.6f}; loss rel bf16 {rel[False]:.2e} fp8 {rel[True]:.2e}; LoRA grad rel bf16 "
          f"{grel[False]:.3e} fp8 {grel[True]:.3e}")
    assert den > 0
    assert rel[False] < 2e-2 and grel[False] < 1e-1
    assert rel[True] < 5e-3 and grel[True] < 5e-2
