"""Is the LoRA effect delta = eps_pol - eps_ref of the HIP paired pass biased against the fp32 oracle?

tools/c2_window_diag.py showed the per-image log-ratio Delta (which grows with |delta|^2) of our path ~1 % off the fp32
one in the same direction on every image, while torch-bf16's is ~0.2 % off: a scale error, not noise.  Here: ONE
input batch at 1024^2, LoRA B non-zero on one adapter group at a time, and for each path (ours, torch-bf16) the
projection coefficients
    rho_eps   = <eps_x - eps_32, eps_32> / |eps_32|^2        (a global scale error of eps)
    rho_delta = <delta_x - delta_32, delta_32> / |delta_32|^2 (a scale error of the LoRA effect)
and the relative distance of delta.  usage (GPU): python tools/lora_bias_diag.py [h] [b_std]"""
import os
import sys
from types import SimpleNamespace

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import sdxl_ref  # noqa: E402
from pairwise_sample_optimization_amd import kernels as K  # noqa: E402
from pairwise_sample_optimization_amd.trainer import compute_time_ids  # noqa: E402
from pairwise_sample_optimization_amd.unet import UNet2DConditionModel, UNetConfig  # noqa: E402


def main():
    h = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    b_std = float(sys.argv[2]) if len(sys.argv) > 2 else 1.5e-2
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    only = sys.argv[4].split(",") if len(sys.argv) > 4 else None
    print(f"oracle precision flags: cudnn.allow_tf32={torch.backends.cudnn.allow_tf32} "
          f"matmul.allow_tf32={torch.backends.cuda.matmul.allow_tf32} "
          f"float32_matmul_precision={torch.get_float32_matmul_precision()}", flush=True)
    if os.environ.get("NO_TF32") == "1":
        torch.backends.cudnn.allow_tf32 = False
        torch.backends.cuda.matmul.allow_tf32 = False
        print("  -> tf32 disabled", flush=True)
    cuda = torch.device("cuda", 0)
    cfg = UNetConfig.sdxl(h)
    with torch.device(cuda):
        unet = UNet2DConditionModel(cfg)
    unet.init_weights(0)
    unet.add_adapter(SimpleNamespace(r=32, lora_alpha=32))
    unet.lora.init_gaussian(seed=0, b_std=b_std)
    unet.prepare()
    full = unet.lora.state_dict_peft()
    sd = sdxl_ref.sd_to(unet.state_dict(), cuda)
    sd16 = {k: v.bfloat16() for k, v in sd.items()}
    ocfg = dict(time_proj_dim=cfg.time_proj_dim, addition_time_embed_dim=cfg.addition_time_embed_dim)
    g = torch.Generator(device="cuda").manual_seed(5)
    x = (torch.randn(n, h, h, 4, device=cuda, generator=g) * 14.6 * 0.0683).bfloat16()
    t = torch.full((n,), 999.0, device=cuda)
    enc = torch.randn(n, 77, 2048, device=cuda, generator=g).bfloat16()
    pooled = torch.randn(n, 1280, device=cuda, generator=g).bfloat16()
    tid = compute_time_ids(8 * h, 0, cuda).repeat(n, 1)
    x_in = K.nhwc_to_nchw(x).float()

    def fwd(wts, lo):
        return torch.cat([sdxl_ref.unet_forward(wts, x_in[i:i + 1], t[i:i + 1], enc[i:i + 1].float(),
                                                pooled[i:i + 1].float(), tid[i:i + 1], lora=lo, cfg=ocfg)
                          for i in range(n)])

    with torch.no_grad():
        er32 = fwd(sd, None)
        if os.environ.get("CPU_CHECK") == "1":  # is the GPU-resident fp32 oracle true fp32?  (CPU fp32 as the judge)
            torch.set_num_threads(16)
            sdc = {k: v.cpu() for k, v in sd.items()}
            ec = sdxl_ref.unet_forward(sdc, x_in[:1].cpu(), t[:1].cpu(), enc[:1].float().cpu(), pooled[:1].float().cpu(),
                                       tid[:1].cpu(), lora=None, cfg=ocfg)
            print(f"fp32 oracle GPU vs CPU (1 image, no LoRA): rel {((er32[:1].cpu() - ec).norm() / ec.norm()).item():.3e}",
                  flush=True)
            del sdc
        with torch.autocast("cuda", dtype=torch.bfloat16):
            er16 = fwd(sd16, None).float()
    q = lambda v: v.bfloat16().float()
    rho = lambda a, b: (((a - b) * b).sum() / (b * b).sum()).item()
    rel = lambda a, b: ((a - b).norm() / b.norm()).item()
    groups = {
        "all": lambda k: True,
        "attn1.qkv": lambda k: ".attn1.to_" in k and "to_out" not in k,
        "attn1.out": lambda k: ".attn1.to_out" in k,
        "attn2.q": lambda k: ".attn2.to_q" in k,
        "attn2.kv": lambda k: ".attn2.to_k" in k or ".attn2.to_v" in k,
        "attn2.out": lambda k: ".attn2.to_out" in k,
        "down": lambda k: k.startswith("down_blocks"),
        "mid": lambda k: k.startswith("mid_block"),
        "up": lambda k: k.startswith("up_blocks"),
        "one block (down_blocks.1.attentions.0.tb0)": lambda k: k.startswith("down_blocks.1.attentions.0.transformer_blocks.0."),
    }
    for name, sel in groups.items():
        if only is not None and name not in only:
            continue
        sdl = {k: (v if (".lora_A." in k or sel(k)) else torch.zeros_like(v)) for k, v in full.items()}
        unet.lora.load_peft(sdl)
        with torch.no_grad():
            eb, _ = unet.forward_nhwc(x, t, enc, pooled, tid, save=False, paired_ref=True)
            lo = {k: v.float() for k, v in sdl.items()}
            ep32 = fwd(sd, lo)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                ep16 = fwd(sd16, lo).float()
        epo, ero = K.nhwc_to_nchw(eb[:n]), K.nhwc_to_nchw(eb[n:])
        d32 = q(ep32) - q(er32)
        do, d16 = epo - ero, q(ep16) - q(er16)
        print(f"{name:44s} |delta|/|eps| {(d32.norm() / ep32.norm()).item():.3e} | ours: rho_eps pol "
              f"{rho(epo, q(ep32)):+.2e} ref {rho(ero, q(er32)):+.2e} rho_delta {rho(do, d32):+.3e} delta rel "
              f"{rel(do, d32):.3e} | torch-bf16: rho_eps pol {rho(q(ep16), q(ep32)):+.2e} ref "
              f"{rho(q(er16), q(er32)):+.2e} rho_delta {rho(d16, d32):+.3e} delta rel {rel(d16, d32):.3e}", flush=True)


if __name__ == "__main__":
    main()
