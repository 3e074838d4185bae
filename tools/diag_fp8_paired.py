"""Diagnostic: does the LoRA act in the paired pass with the fp8 forward on?  (sdxl32; prints the policy-vs-reference
eps distance of the paired pass and of separate LoRA-on / LoRA-off passes, bf16 and fp8.)"""
import os
import sys
from types import SimpleNamespace

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pairwise_sample_optimization_amd.unet import UNet2DConditionModel, UNetConfig  # noqa: E402

dev = torch.device("cuda", 0)
for h in (32, 64):
    cfg = UNetConfig.sdxl(h)
    with torch.device(dev):
        unet = UNet2DConditionModel(cfg)
    unet.init_weights(0)
    unet.add_adapter(SimpleNamespace(r=16, lora_alpha=16))
    unet.lora.init_gaussian(seed=1, b_std=2e-2)
    unet.prepare()
    g = torch.Generator(device="cuda").manual_seed(3)
    n = 2
    x = torch.randn(n, h, h, 4, device=dev, generator=g).bfloat16()
    t = torch.full((n,), 999.0, device=dev)
    enc = torch.randn(n, 77, 2048, device=dev, generator=g).bfloat16()
    pooled = torch.randn(n, 1280, device=dev, generator=g).bfloat16()
    tid = torch.tensor([[8 * h, 8 * h, 0, 0, 8 * h, 8 * h]], device=dev, dtype=torch.float32).repeat(n, 1)
    for fp8 in (False, True):
        unet.enable_fp8_forward(fp8)
        with torch.no_grad():
            e2, _ = unet.forward_nhwc(x, t, enc, pooled, tid, save=False, paired_ref=True)
            on, _ = unet.forward_nhwc(x, t, enc, pooled, tid, save=False)
            unet.disable_adapters()
            off, _ = unet.forward_nhwc(x, t, enc, pooled, tid, save=False)
            unet.enable_adapters()
        rel = lambda a, b: ((a.float() - b.float()).norm() / b.float().norm()).item()
        print(f"h={h} fp8={fp8}: paired pol-ref {rel(e2[:n], e2[n:]):.3e}; separate on-off {rel(on, off):.3e}; "
              f"paired pol vs separate on {rel(e2[:n], on):.3e}; paired ref vs off {rel(e2[n:], off):.3e}", flush=True)
