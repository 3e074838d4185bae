"""Split-count sweep of the TN GEMM (LoRA weight gradients) and timing of the skinny-N GEMM on UNet shapes."""
import os
os.environ.setdefault("PSO_LIB", "knobs")  # benchmark knobs: the tools build (include/pso_amd_knobs.h)
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pairwise_sample_optimization_amd import kernels as K  # noqa: E402
from tools.gemm_bench import t_ms  # noqa: E402


def main():
    dev = torch.device("cuda")
    for (M, I, J) in [(8192, 1280, 32), (8192, 32, 1280), (8192, 96, 1280), (32768, 640, 32), (616, 1280, 32),
                      (616, 64, 2048), (32768, 32, 640)]:
        a = torch.randn(M, I, device=dev).bfloat16()
        b = torch.randn(M, J, device=dev).bfloat16()
        out = torch.zeros(I, J, device=dev)
        line = []
        for ks in ((0,) if os.environ.get("TN_ONLY_AUTO") else (0, 1, 2, 4, 8, 16, 32, 64)):
            K.lib().pso_gemm_tn_set_split(ks)
            line.append(f"ks{ks}={t_ms(lambda: K.gemm_tn(a, b, out)) * 1e3:7.1f}us")
        K.lib().pso_gemm_tn_set_split(0)
        print(f"tn {M}x{I}x{J}: " + " ".join(line))
    for (M, N, Kd) in [(8192, 32, 1280), (8192, 96, 1280), (32768, 32, 640), (616, 32, 1280), (616, 64, 2048),
                       (131072, 32, 320)]:
        a = torch.randn(M, Kd, device=dev).bfloat16()
        w = torch.randn(N, Kd, device=dev).bfloat16()
        us = t_ms(lambda: K.gemm(a, w)) * 1e3
        print(f"skinny {M}x{N}x{Kd}: {us:7.1f} us  {M * Kd * 2 / us / 1e3:7.1f} GB/s (A stream)")


if __name__ == "__main__":
    main()
