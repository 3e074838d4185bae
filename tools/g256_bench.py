"""Where the 8-phase kernels lose to the vendor library on the UNet's big GEMMs: per shape, the dispatched kernel with
and without its epilogue (main loop alone), against torch.matmul (hipBLASLt) on the same operands.
usage: python tools/g256_bench.py  (GPU; GEMM_VARIANTS=0,39 to add dispatch variants)"""
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
    shapes = [(4096, 4096, 4096), (8192, 8192, 8192), (16384, 10240, 1280), (8192, 10240, 1280),
              (16384, 3840, 1280), (8192, 1280, 10240), (16384, 1280, 5120), (8192, 5120, 1280),
              (65536, 5120, 640), (16384, 1280, 1280)]
    variants = [int(v) for v in os.environ.get("GEMM_VARIANTS", "0").split(",")]
    for M, N, Kd in shapes:
        a = torch.randn(M, Kd, device=dev).bfloat16()
        w = torch.randn(N, Kd, device=dev).bfloat16()
        fl = 2 * M * N * Kd
        res = []
        for v in variants:
            K.gemm_set_variant(v)
            for skip in (0, 1):
                K.lib().pso_gemm8p_skip_epilogue(skip)
                ms = t_ms(lambda: K.gemm(a, w))
                kn = K.lib().pso_last_kernel().decode()
                res.append(f"v{v}{'-loop' if skip else ''} {fl / ms / 1e9:6.0f}")
            K.lib().pso_gemm8p_skip_epilogue(0)
        K.gemm_set_variant(0)
        ms = t_ms(lambda: a @ w.t())
        res.append(f"hipBLASLt {fl / ms / 1e9:6.0f}")
        print(f"{M}x{N}x{Kd} [{kn}]: " + " | ".join(res) + " TF/s", flush=True)
    # ff.out as the step runs it: bias + residual epilogue
    M, N, Kd = 16384, 1280, 5120
    a = torch.randn(M, Kd, device=dev).bfloat16()
    w = torch.randn(N, Kd, device=dev).bfloat16()
    b = torch.randn(N, device=dev).bfloat16()
    r = torch.randn(M, N, device=dev).bfloat16()
    fl = 2 * M * N * Kd
    for v in variants:
        K.gemm_set_variant(v)
        res = []
        for name, kw in (("plain", {}), ("bias", dict(bias=b)), ("bias+resid", dict(bias=b, resid=r))):
            ms = t_ms(lambda: K.gemm(a, w, **kw))
            res.append(f"{name} {fl / ms / 1e9:6.0f}")
        print(f"ff.out {M}x{N}x{Kd} v{v} [{K.lib().pso_last_kernel().decode()}]: " + " | ".join(res) + " TF/s",
              flush=True)
    K.gemm_set_variant(0)
    # the GEGLU projection (fused epilogue, pre-activation saved for half the rows as in the paired pass)
    for M, N, Kd in [(16384, 10240, 1280), (65536, 5120, 640)]:
        a = torch.randn(M, Kd, device=dev).bfloat16()
        w = torch.randn(N, Kd, device=dev).bfloat16()
        b = torch.randn(N, device=dev).bfloat16()
        pre = torch.empty(M // 2, N, device=dev).bfloat16()
        fl = 2 * M * N * Kd
        res = []
        for skip in (0, 1):
            K.lib().pso_gemm8p_skip_epilogue(skip)
            ms = t_ms(lambda: K.gemm_geglu(a, w, b, out_pre=pre, pre_rows=M // 2))
            res.append(f"{'loop' if skip else 'geglu'} {fl / ms / 1e9:6.0f}")
        K.lib().pso_gemm8p_skip_epilogue(0)
        print(f"GEGLU {M}x{N}x{Kd} [{K.lib().pso_last_kernel().decode()}]: " + " | ".join(res) + " TF/s", flush=True)


if __name__ == "__main__":
    main()
