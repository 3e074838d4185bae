"""Is the 8-phase GEMM's epilogue bound per CU (store issue) or chip-wide (HBM writes)?  One round of 256x256 tiles
(K = 1280) on 32 / 64 / 128 / 256 CUs, with and without the epilogue: the per-tile epilogue time stays flat with the
CU count when each CU's store stream is the limit, and grows with it when the chip's write bandwidth is.
usage: python tools/epi_rate.py  (GPU)"""
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
    Kd = 1280
    K.gemm_set_variant(30)  # 256 x 256 8-phase wherever it applies
    for tiles in (32, 64, 128, 256, 512):
        M, N = 256 * tiles // 4, 1024
        a = torch.randn(M, Kd, device=dev).bfloat16()
        w = torch.randn(N, Kd, device=dev).bfloat16()
        r = torch.randn(M, N, device=dev).bfloat16()
        out = {}
        for name, kw in (("plain", {}), ("resid", dict(resid=r))):
            for skip in (0, 1):
                K.lib().pso_gemm8p_skip_epilogue(skip)
                out[(name, skip)] = t_ms(lambda: K.gemm(a, w, **kw), it=50) * 1e3
            K.lib().pso_gemm8p_skip_epilogue(0)
        kn = K.lib().pso_last_kernel().decode()
        rounds = (tiles + 255) // 256
        print(f"{tiles:4d} tiles ({rounds} round) [{kn}]: loop {out[('plain', 1)]:7.1f} us | plain epilogue "
              f"{(out[('plain', 0)] - out[('plain', 1)]) / rounds:6.1f} us/round | +resid "
              f"{(out[('resid', 0)] - out[('resid', 1)]) / rounds:6.1f} us/round", flush=True)
    K.gemm_set_variant(0)


if __name__ == "__main__":
    main()
