"""fp8 (scaled e4m3 MFMA) vs bf16 GEMM on the UNet's LayerNorm-fed projections (q/k/v, cross q, GEGLU proj), plus the
row quantisation pass the fp8 path adds in front of each.  usage: FP8_IMAGES=8 python tools/fp8_bench.py   (GPU)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pairwise_sample_optimization_amd import kernels as K  # noqa: E402
from tools.gemm_bench import t_ms  # noqa: E402


def main():
    dev = torch.device("cuda")
    x = torch.randn(8192, 8192, device=dev).bfloat16()
    for _ in range(200):
        x @ x
    torch.cuda.synchronize()
    Bi = int(os.environ.get("FP8_IMAGES", "8"))
    L1, L2 = 4096 * Bi, 1024 * Bi
    shapes = [(4096, 4096, 4096, "square", False), (L2, 3840, 1280, "L2 qkv", False), (L2, 1280, 1280, "L2 q2", False),
              (L2, 10240, 1280, "L2 ff.proj (GEGLU)", True), (L1, 5120, 640, "L1 ff.proj (GEGLU)", True)]
    for M, N, Kd, name, geglu in shapes:
        a = torch.randn(M, Kd, device=dev).bfloat16()
        w = (torch.randn(N, Kd, device=dev) / Kd ** 0.5).bfloat16()
        b = torch.randn(N, device=dev).bfloat16()
        wa = K.quant_rows_fp8(w)
        aq = K.quant_rows_fp8(a)
        if geglu:
            bf = t_ms(lambda: K.gemm_geglu(a, w, b))
            f8 = t_ms(lambda: K.gemm_fp8(aq, wa, bias=b, geglu=True))
        else:
            bf = t_ms(lambda: K.gemm(a, w, bias=b))
            f8 = t_ms(lambda: K.gemm_fp8(aq, wa, bias=b))
        qt = t_ms(lambda: K.quant_rows_fp8(a, q=aq[0], e=aq[1]))
        fl = 2.0 * M * N * Kd
        print(f"{name:22s} {M}x{N}x{Kd}: bf16 {bf:.3f} ms {fl / bf / 1e9:6.0f} TF/s | fp8 {f8:.3f} ms "
              f"{fl / f8 / 1e9:6.0f} TF/s | quant {qt * 1e3:6.1f} us ({3.0 * M * Kd / qt / 1e6:5.0f} GB/s) | "
              f"fp8+quant {fl / (f8 + qt) / 1e9:6.0f} TF/s", flush=True)


if __name__ == "__main__":
    main()
