"""GroupNorm / LayerNorm kernels on the C2 step's shapes: per-kernel time (rocprofv3 splits a call into its partial /
finalize / apply launches) and the call's algorithmic bytes -> GB/s.  usage (GPU): python tools/norm_bench.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pairwise_sample_optimization_amd import kernels as K  # noqa: E402


def t_us(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


def main():
    dev = torch.device("cuda")
    torch.manual_seed(0)
    print("GroupNorm (NHWC, 32 groups)          fwd us  GB/s | bwd us  GB/s   (fwd: x in, y out; bwd: x, dy in, dx out)")
    for B, H, C, silu in [(16, 128, 320, True), (16, 64, 640, True), (16, 32, 1280, True), (8, 64, 640, True),
                          (16, 64, 640, False), (8, 128, 640, True)]:
        x = torch.randn(B, H, H, C, device=dev).bfloat16()
        gm = (1 + 0.1 * torch.randn(C, device=dev)).bfloat16()
        bt = (0.1 * torch.randn(C, device=dev)).bfloat16()
        y, st = K.group_norm_fwd(x, gm, bt, 32, 1e-5, silu)
        dy = torch.randn_like(x)
        nb = x.numel() * 2
        tf = t_us(lambda: K.group_norm_fwd(x, gm, bt, 32, 1e-5, silu))
        tb = t_us(lambda: K.group_norm_bwd(x, dy, st, gm, bt, silu))
        print(f"B{B:3d} {H}x{H}x{C:5d} silu={int(silu)}            {tf:7.1f} {2 * nb / tf / 1e3:6.0f} | "
              f"{tb:7.1f} {3 * nb / tb / 1e3:6.0f}", flush=True)
    x = torch.randn(16, 128, 128, 320, device=dev).bfloat16()
    y = torch.empty_like(x)
    tc = t_us(lambda: y.copy_(x))
    print(f"torch copy of 16x128x128x320 bf16 (reference streaming rate): {tc:.1f} us {2 * x.numel() * 2 / tc / 1e3:.0f} GB/s")
    print("LayerNorm                            fwd us  GB/s | bwd us  GB/s")
    for M, C in [(16384, 1280), (65536, 640), (8192, 1280), (32768, 640), (4096, 1280)]:
        x = torch.randn(M, C, device=dev).bfloat16()
        gm = (1 + 0.1 * torch.randn(C, device=dev)).bfloat16()
        bt = (0.1 * torch.randn(C, device=dev)).bfloat16()
        y, st = K.layer_norm_fwd(x, gm, bt, 1e-5)
        dy = torch.randn_like(x)
        nb = x.numel() * 2
        tf = t_us(lambda: K.layer_norm_fwd(x, gm, bt, 1e-5))
        tb = t_us(lambda: K.layer_norm_bwd(x, dy, st, gm))
        print(f"{M:6d} x {C:5d}                       {tf:7.1f} {2 * nb / tf / 1e3:6.0f} | "
              f"{tb:7.1f} {3 * nb / tb / 1e3:6.0f}", flush=True)


if __name__ == "__main__":
    main()
