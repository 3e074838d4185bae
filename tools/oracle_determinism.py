"""Is the torch-bf16 yardstick of the parity windows (oracle/sdxl_ref.py under bf16 autocast) deterministic?  Runs the
1024^2 UNet forward of one image twice per setting and compares the bits; settings: default, and
torch.backends.cudnn.deterministic = True (MIOpen's deterministic algorithms).  usage (GPU): python tools/oracle_determinism.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import sdxl_ref  # noqa: E402
from pairwise_sample_optimization_amd import kernels as K  # noqa: E402
from pairwise_sample_optimization_amd.trainer import compute_time_ids  # noqa: E402
from pairwise_sample_optimization_amd.unet import UNet2DConditionModel, UNetConfig  # noqa: E402


def main():
    cuda = torch.device("cuda", 0)
    cfg = UNetConfig.sdxl(128)
    with torch.device(cuda):
        unet = UNet2DConditionModel(cfg)
    unet.init_weights(0)
    sd = sdxl_ref.sd_to(unet.state_dict(), cuda)
    sd16 = {k: v.bfloat16() for k, v in sd.items()}
    ocfg = dict(time_proj_dim=cfg.time_proj_dim, addition_time_embed_dim=cfg.addition_time_embed_dim)
    g = torch.Generator(device="cuda").manual_seed(5)
    x = (torch.randn(1, 4, 128, 128, device=cuda, generator=g) * 0.9)
    t = torch.full((1,), 999.0, device=cuda)
    enc = torch.randn(1, 77, 2048, device=cuda, generator=g)
    pooled = torch.randn(1, 1280, device=cuda, generator=g)
    tid = compute_time_ids(1024, 0, cuda)

    def f16():
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
            return sdxl_ref.unet_forward(sd16, x, t, enc, pooled, tid, lora=None, cfg=ocfg).float()

    def f32():
        with torch.no_grad():
            return sdxl_ref.unet_forward(sd, x, t, enc, pooled, tid, lora=None, cfg=ocfg)

    import time

    def timed(fn, n=2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            out = fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n, out

    def bwd32():
        xi = x.clone().requires_grad_(True)
        out = sdxl_ref.unet_forward(sd, xi, t, enc, pooled, tid, lora=None, cfg=ocfg)
        out.sum().backward()
        return xi.grad

    for det in (False, True):
        torch.backends.cudnn.deterministic = det
        f16()
        f32()
        tf16, a = timed(f16)
        tf32, d = timed(f32)
        tb32, _ = timed(bwd32, 1)
        print(f"cudnn.deterministic={det}: bf16 fwd {tf16:.3f} s, fp32 fwd {tf32:.3f} s, fp32 fwd+bwd {tb32:.3f} s",
              flush=True)
        b, c = f16(), f16()
        e = f32()
        print(f"cudnn.deterministic={det}: bf16 run-to-run identical {torch.equal(a, b)} / {torch.equal(a, c)} "
              f"(max |diff| {(a - b).abs().max().item():.3e}); fp32 identical {torch.equal(d, e)} "
              f"(max |diff| {(d - e).abs().max().item():.3e}); bf16 rel to fp32 {((a - d).norm() / d.norm()).item():.4e}",
              flush=True)


if __name__ == "__main__":
    main()
