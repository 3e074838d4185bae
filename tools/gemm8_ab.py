"""Same-process A/B of the 8-phase 256x256 GEMM modes (pso_gemm8p_skip_epilogue bit 1 = staggered wave groups) on the
UNet's N % 256 shapes, interleaved rounds, with a max-error check of each mode against an fp32 product.  (GPU)"""
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
    mode = lib.pso_gemm8p_skip_epilogue
    mode.argtypes = [ctypes.c_int]
    x = torch.randn(8192, 8192, device=dev).bfloat16()
    for _ in range(200):
        x @ x
    torch.cuda.synchronize()
    modes = [int(m) for m in os.environ.get("MODES", "0").split(",")]
    shapes = [(4096, 4096, 4096, "square"), (16384, 3840, 1280, "L2 qkv x16"), (16384, 1280, 5120, "L2 ffout x16"),
              (8192, 1280, 10240, "L2 geglu dX x8"), (16384, 1280, 1280, "L2 proj x16"), (8192, 5120, 1280, "ffout dX")]
    for M, N, Kd, name in shapes:
        a = torch.randn(M, Kd, device=dev).bfloat16()
        w = torch.randn(N, Kd, device=dev).bfloat16()
        ref = a.float() @ w.float().t()
        res = {m: [] for m in modes + ["auto"]}
        for r in range(3):
            K.gemm_set_variant(0)
            res["auto"].append(t_ms(lambda: K.gemm(a, w)))
            K.gemm_set_variant(30)
            for m in modes:
                mode(m)
                res[m].append(t_ms(lambda: K.gemm(a, w)))
        errs = {}
        for m in modes:
            mode(m)
            errs[m] = ((K.gemm(a, w).float() - ref).abs().max() / ref.abs().max()).item()
        fl = 2 * M * N * Kd
        print(f"{name:16s} {M}x{N}x{Kd}: auto {fl / min(res['auto']) / 1e9:6.0f} TF/s  " + "  ".join(
            f"mode {m}: {fl / min(res[m]) / 1e9:6.0f} TF/s (err {errs[m]:.1e})" for m in modes), flush=True)
    for (M, F, Kd, name) in [(16384, 5120, 1280, "L2x2 geglu"), (65536, 2560, 640, "L1x2 geglu")]:
        a = torch.randn(M, Kd, device=dev).bfloat16()
        w = (torch.randn(2 * F, Kd, device=dev) / Kd ** 0.5).bfloat16()
        b = torch.randn(2 * F, device=dev).bfloat16()
        pre = torch.empty(M // 2, 2 * F, device=dev, dtype=torch.bfloat16)
        K.gemm_set_variant(0)
        res = {m: [] for m in modes}
        outs = {}
        for r in range(3):
            for m in modes:
                mode(m)
                res[m].append(t_ms(lambda: K.gemm_geglu(a, w, b, out_pre=pre, pre_rows=M // 2)))
        for m in modes:
            mode(m)
            o = K.gemm_geglu(a, w, b, out_pre=pre, pre_rows=M // 2)
            outs[m] = (o[0] if isinstance(o, tuple) else o).float()
        fl = 2 * M * 2 * F * Kd
        d = max((outs[m] - outs[modes[0]]).abs().max().item() for m in modes)
        print(f"{name:16s} {M}x{2 * F}x{Kd}: " + "  ".join(
            f"mode {m}: {fl / min(res[m]) / 1e9:6.0f} TF/s" for m in modes) + f"  maxdiff {d:.1e}", flush=True)
    for (M, F, Kd, name) in [(8192, 5120, 1280, "L2 geglu bwd"), (32768, 2560, 640, "L1 geglu bwd")]:
        dy = torch.randn(M, Kd, device=dev).bfloat16()
        wt = (torch.randn(F, Kd, device=dev) / Kd ** 0.5).bfloat16()
        pre = torch.randn(M, 2 * F, device=dev).bfloat16()
        res = {v: [] for v in (0, 30)}
        outs = {}
        mode(0)
        for r in range(3):
            for v in res:
                K.gemm_set_variant(v)
                res[v].append(t_ms(lambda: K.gemm_geglu_bwd(dy, wt, pre)))
        for v in res:
            K.gemm_set_variant(v)
            outs[v] = K.gemm_geglu_bwd(dy, wt, pre).float()
        fl = 2 * M * F * Kd
        print(f"{name:16s} {M}x{F}x{Kd}: " + "  ".join(f"variant {v}: {fl / min(res[v]) / 1e9:6.0f} TF/s" for v in res)
              + f"  maxdiff {(outs[30] - outs[0]).abs().max().item():.1e}", flush=True)
    mode(0)
    K.gemm_set_variant(0)


if __name__ == "__main__":
    main()
