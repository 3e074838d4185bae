"""What the fused epilogue terms and the LoRA K-tail cost on the short-K projection GEMMs of the paired pass
(M=16384 / 8192, N=1280, K=1280): plain / +bias / +bias+resid / +LoRA tail / +tail limited to the policy rows.
EPI_FLUSH=1 streams a 512 MB buffer between launches so every operand comes from HBM as in the train step."""
import os
os.environ.setdefault("PSO_LIB", "knobs")  # benchmark knobs: the tools build (include/pso_amd_knobs.h)
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pairwise_sample_optimization_amd import kernels as K  # noqa: E402


def main():
    dev = torch.device("cuda")
    flush = torch.empty(256 << 20, dtype=torch.bfloat16, device=dev) if os.environ.get("EPI_FLUSH") else None
    for v in [int(x) for x in os.environ.get("GEMM_VARIANTS", "0").split(",")]:
        K.gemm_set_variant(v)
        print(f"--- variant {v} flush={flush is not None} ---")
        for M, N, Kd, r in [(16384, 1280, 1280, 32), (8192, 1280, 1280, 32), (65536, 640, 640, 32)]:
            a = torch.randn(M, Kd, device=dev).bfloat16()
            w = torch.randn(N, Kd, device=dev).bfloat16()
            bias = torch.randn(N, device=dev).bfloat16()
            res = torch.randn(M, N, device=dev).bfloat16()
            a2 = torch.randn(M // 2, r, device=dev).bfloat16()
            a2f = torch.randn(M, r, device=dev).bfloat16()
            w2 = torch.randn(N, r, device=dev).bfloat16()
            out = torch.empty(M, N, device=dev).bfloat16()
            cases = [("plain", dict()), ("bias", dict(bias=bias)), ("bias+resid", dict(bias=bias, resid=res)),
                     ("tail(all rows)", dict(a2=a2f, w2=w2)), ("tail(half rows)", dict(a2=a2, w2=w2, tail_rows=M // 2)),
                     ("all", dict(bias=bias, resid=res, a2=a2, w2=w2, tail_rows=M // 2))]
            for name, kw in cases:
                fn = lambda: K.gemm(a, w, out=out, **kw)  # noqa: E731
                for _ in range(3):
                    fn()
                torch.cuda.synchronize()
                tot = 0.0
                it = 20
                for _ in range(it):
                    if flush is not None:
                        flush.zero_()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    fn()
                    e1.record()
                    torch.cuda.synchronize()
                    tot += e0.elapsed_time(e1)
                ms = tot / it
                print(f"{M}x{N}x{Kd} {name:16s} {ms * 1e3:8.1f} us  {2 * M * N * Kd / ms / 1e9:7.1f} TF/s")


if __name__ == "__main__":
    main()
