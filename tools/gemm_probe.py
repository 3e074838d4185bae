"""GEMM cost model probe (GPU): for the UNet's dominant shapes, time the default dispatch, the 8-phase 256x256 kernel
with and without its epilogue stores, and the 8-phase kernel at K, 2K, 4K (per-K-tile cost and fixed per-tile cost),
plus hipBLASLt (torch.mm) for reference.  Random bf16 operands."""
import ctypes
import os
os.environ.setdefault("PSO_LIB", "knobs")  # benchmark knobs: the tools build (include/pso_amd_knobs.h)
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pairwise_sample_optimization_amd import kernels as K  # noqa: E402
from tools.gemm_bench import t_ms  # noqa: E402


def main():
    dev = torch.device("cuda")
    lib = K.lib()
    skip = lib.pso_gemm8p_skip_epilogue
    skip.argtypes = [ctypes.c_int]
    x = torch.randn(8192, 8192, device=dev).bfloat16()
    for _ in range(200):
        x @ x
    torch.cuda.synchronize()
    shapes = [(4096, 4096, 4096, "square"), (16384, 3840, 1280, "L2 qkv x16"), (16384, 10240, 1280, "L2 ffproj x16"),
              (8192, 5120, 1280, "L2 ffout dX x8"), (65536, 5120, 640, "L1 ffproj x16"), (16384, 1280, 5120, "L2 ffout x16"),
              (16384, 1280, 1280, "L2 proj x16"), (65536, 1920, 640, "L1 qkv x16"), (65536, 640, 640, "L1 proj x16")]
    for M, N, Kd, name in shapes:
        res = []
        for kk in (1, 2, 4):
            Kx = Kd * kk
            a = torch.randn(M, Kx, device=dev).bfloat16()
            w = torch.randn(N, Kx, device=dev).bfloat16()
            fl = 2 * M * N * Kx
            K.gemm_set_variant(0)
            t0 = t_ms(lambda: K.gemm(a, w))
            row = [f"K={Kx}: auto {fl / t0 / 1e9:6.0f}"]
            if N % 256 == 0:
                K.gemm_set_variant(30)
                t1 = t_ms(lambda: K.gemm(a, w))
                skip(1)
                t2 = t_ms(lambda: K.gemm(a, w))
                skip(0)
                row.append(f"8p {fl / t1 / 1e9:6.0f} 8p-noepi {fl / t2 / 1e9:6.0f} (epi {1e3 * (t1 - t2):6.1f} us)")
            wt = w.t()
            t3 = t_ms(lambda: torch.mm(a, wt))
            row.append(f"hipBLASLt {fl / t3 / 1e9:6.0f}")
            res.append("  ".join(row))
            K.gemm_set_variant(0)
            if kk == 1 and M * Kd > 65536 * 1280:
                break
        print(f"{name} {M}x{N}x{Kd}:")
        for r in res:
            print("    " + r)
        sys.stdout.flush()


if __name__ == "__main__":
    main()
