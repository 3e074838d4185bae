"""The SDXL VAE decoder's 3x3 convolutions (one 4-image chunk at 1024^2, vae.py _decode_chunk) under every forced
tile variant of the GEMM dispatch (knobs build): TF/s per shape, to pick the tile rule for the N % 160 != 0 widths
(128 / 256 / 512 channels).  usage (GPU): GEMM_VARIANTS=0,1,2,3,4,5,7,8,28 python tools/vae_conv_bench.py"""
import os
os.environ.setdefault("PSO_LIB", "knobs")  # benchmark knobs: the tools build (include/pso_amd_knobs.h)
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pairwise_sample_optimization_amd import kernels as K  # noqa: E402

# (latent side, Cin, Cout, mode): per 4-image chunk; the count is the number of such convs per chunk
SHAPES = [(128, 512, 512, K.CONV_NORMAL, 10), (256, 512, 512, K.CONV_UP2, 1), (256, 512, 512, K.CONV_NORMAL, 6),
          (512, 512, 512, K.CONV_UP2, 1), (512, 512, 256, K.CONV_NORMAL, 1), (512, 256, 256, K.CONV_NORMAL, 5),
          (1024, 256, 256, K.CONV_UP2, 1), (1024, 256, 128, K.CONV_NORMAL, 1), (1024, 128, 128, K.CONV_NORMAL, 5)]


def t_ms(fn, it=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it


def main():
    dev = torch.device("cuda")
    variants = [int(v) for v in os.environ.get("GEMM_VARIANTS", "0,1,2,3,4,5,7,8,28").split(",")]
    print("shape (side Cin->Cout mode x count)".ljust(40) + "".join(f"{'v' + str(v):>8}" for v in variants) +
          "   (TF/s; ms per chunk for v0)")
    tot = {v: 0.0 for v in variants}
    for side, cin, cout, mode, cnt in SHAPES:
        hin = side // 2 if mode == K.CONV_UP2 else side
        g = torch.Generator(device="cuda").manual_seed(side + cin + cout)
        x = torch.randn(4, hin, hin, cin, device=dev, generator=g).bfloat16()
        w = (torch.randn(cout, 3, 3, cin, device=dev, generator=g) / (9 * cin) ** 0.5).bfloat16()
        b = (0.1 * torch.randn(cout, device=dev, generator=g)).bfloat16()
        fl = 2.0 * 4 * side * side * cout * 9 * cin
        line = f"{side}^2 {cin}->{cout} {'up2' if mode == K.CONV_UP2 else 'n'} x{cnt}".ljust(40)
        ref = None
        for v in variants:
            K.gemm_set_variant(v)
            try:
                y = K.conv2d(x, w, mode=mode, bias=b)
                if ref is None:
                    ref = y.float()
                err = ((y.float() - ref).norm() / ref.norm()).item()
                ms = t_ms(lambda: K.conv2d(x, w, mode=mode, bias=b))
                tot[v] += ms * cnt
                line += f"{fl / ms / 1e9:7.0f}{'!' if err > 1e-2 else ' '}"
            except Exception:
                tot[v] += float("nan")
                line += f"{'-':>7} "
        K.gemm_set_variant(0)
        K.conv2d(x, w, mode=mode, bias=b)
        line += "  " + K.lib().pso_last_kernel().decode().replace("gemm_bf16_kernel", "2p").replace("gemm8p_kernel", "8p")
        print(line, flush=True)
        del x, w, y
        torch.cuda.empty_cache()
    print("ms per chunk (sum over the listed convs)".ljust(40) + "".join(f"{tot[v]:8.2f}" for v in variants))


if __name__ == "__main__":
    main()
