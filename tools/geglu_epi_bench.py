"""GEGLU forward (ff.net.0.proj + gelu gate, the 8-phase 256 x 256 EPI_GEGLU kernel) at the C2 step's shapes: whole
kernel vs main loop alone (skip-epilogue knob), with / without the pre-activation store of the policy rows, and the
same product as a plain GEMM (bf16 out, no gate).  usage (GPU): python tools/geglu_epi_bench.py"""
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
    for _ in range(100):
        x @ x
    for M, C, F in ((65536, 640, 2560), (16384, 1280, 5120)):
        a = torch.randn(M, C, device=dev).bfloat16()
        w = (torch.randn(2 * F, C, device=dev) / C ** 0.5).bfloat16()
        b = torch.randn(2 * F, device=dev).bfloat16()
        pre = torch.empty(M // 2, 2 * F, device=dev).bfloat16()
        fl = 2 * M * 2 * F * C
        row = []
        for name, fn in (("geglu+pre", lambda: K.gemm_geglu(a, w, b, out_pre=pre, pre_rows=M // 2)),
                         ("geglu", lambda: K.gemm_geglu(a, w, b)),
                         ("plain", lambda: K.gemm(a, w, bias=b))):
            for skip in (0, 1):
                K.lib().pso_gemm8p_skip_epilogue(skip)
                ms = t_ms(fn, 20)
                row.append(f"{name}{'-loop' if skip else ''} {ms * 1e3:6.1f} us {fl / ms / 1e9:5.0f} TF/s")
            K.lib().pso_gemm8p_skip_epilogue(0)
        print(f"{M}x{2 * F}x{C}: " + " | ".join(row), flush=True)


if __name__ == "__main__":
    main()
