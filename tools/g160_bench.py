"""Main-loop vs whole-kernel timing of the 8-phase 256 x 160 GEMM against the 2-phase 128 x 160 one on the UNet's
N % 160 shapes at 16 images (variant 37 = 2-phase, 38 = 8-phase; 'loop' = 8-phase with the epilogue skipped).
usage: python tools/g160_bench.py  (GPU)"""
import os
os.environ.setdefault("PSO_LIB", "knobs")  # benchmark knobs: the tools build (include/pso_amd_knobs.h)
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
    shapes = [(16384, 1280, 1280), (8192, 1280, 1280), (65536, 640, 640), (16384, 1280, 5120), (65536, 640, 2560),
              (8192, 1280, 10240), (65536, 1920, 640), (262144, 320, 320)]
    for M, N, Kd in shapes:
        a = torch.randn(M, Kd, device=dev).bfloat16()
        w = torch.randn(N, Kd, device=dev).bfloat16()
        res = []
        for name, v, skip in [("2ph", 37, 0), ("8ph", 38, 0), ("8ph-loop", 38, 1)]:
            K.gemm_set_variant(v)
            K.lib().pso_gemm8p_skip_epilogue(skip)
            ms = t_ms(lambda: K.gemm(a, w))
            res.append(f"{name} {2 * M * N * Kd / ms / 1e9:7.1f}")
        K.lib().pso_gemm8p_skip_epilogue(0)
        K.gemm_set_variant(0)
        print(f"{M}x{N}x{Kd}: " + " | ".join(res) + " TF/s", flush=True)


if __name__ == "__main__":
    main()
