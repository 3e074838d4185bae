"""Micro-benchmark of the MFMA GEMM / implicit-GEMM conv kernel on the SDXL UNet's dominant shapes (1024^2, B=4)."""
import sys
import os
os.environ.setdefault("PSO_LIB", "knobs")  # benchmark knobs: the tools build (include/pso_amd_knobs.h)
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pairwise_sample_optimization_amd import kernels as K  # noqa: E402


def t_ms(fn, it=20):
    for _ in range(3):
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
    x = torch.randn(8192, 8192, device=dev).bfloat16()
    for _ in range(200):  # ~1 s of MFMA work first: clocks settle before the first measured variant
        x @ x
    torch.cuda.synchronize()
    if os.environ.get("GEMM_PREWARM"):  # one silent pass over every shape (first-touch / clock effects)
        run(dev, quiet=True)
    for v in [int(x) for x in os.environ.get("GEMM_VARIANTS", "0").split(",")]:
        K.gemm_set_variant(v)
        print(f"--- variant {v} ---")
        run(dev)


_GEGLU_FIRST = {}


def run(dev, quiet=False):
    torch.manual_seed(0)
    rows = []
    Bi = int(os.environ.get("GEMM_IMAGES", "8"))
    if os.environ.get("GEMM_ONLY_LINEAR"):
        pass
    L1, L2 = 4096 * Bi, 1024 * Bi
    dense = [] if os.environ.get("GEMM_ONLY_GEGLU") else [(4096, 4096, 4096, "square"), (L1, 5120, 640, "L1 ff.proj"),
                             (L1, 640, 2560, "L1 ff.out"), (L1, 1920, 640, "L1 qkv"),
                             (L1, 640, 640, "L1 out/proj"), (L2, 10240, 1280, "L2 ff.proj"),
                             (L2, 1280, 5120, "L2 ff.out"), (L2, 3840, 1280, "L2 qkv"),
                             (L2, 1280, 1280, "L2 proj"), (L2, 1280, 10240, "L2 geglu dX"),
                             (2 * L2, 1280, 5120, "L2x2 ff.out"), (2 * L2, 1280, 1280, "L2x2 proj"),
                             (L2, 5120, 1280, "L2 ff.out dX")]
    for (M, N, Kd, name) in dense:
        a = torch.randn(M, Kd, device=dev).bfloat16()
        w = torch.randn(N, Kd, device=dev).bfloat16()
        ms = t_ms(lambda: K.gemm(a, w))
        ref = a.float() @ w.float().t()
        err = ((K.gemm(a, w).float() - ref).norm() / ref.norm()).item()
        rows.append((name, f"{M}x{N}x{Kd} e={err:.1e}", ms, 2 * M * N * Kd / ms / 1e9))
        if os.environ.get("GEMM_LIB"):  # hipBLASLt (torch.mm) on the same operands, for the headroom column only
            wt = w.t()
            ms = t_ms(lambda: torch.mm(a, wt))
            rows.append(("  hipBLASLt " + name, f"{M}x{N}x{Kd}", ms, 2 * M * N * Kd / ms / 1e9))
    for (M, F, Kd, name) in [(2 * L2, 5120, 1280, "L2x2 geglu"), (2 * L1, 2560, 640, "L1x2 geglu")]:
        a = torch.randn(M, Kd, device=dev).bfloat16()
        w = (torch.randn(2 * F, Kd, device=dev) / Kd ** 0.5).bfloat16()
        b = torch.randn(2 * F, device=dev).bfloat16()
        pre = torch.empty(M // 2, 2 * F, device=dev, dtype=torch.bfloat16)
        ms = t_ms(lambda: K.gemm_geglu(a, w, b, out_pre=pre, pre_rows=M // 2))
        o = K.gemm_geglu(a, w, b, out_pre=pre, pre_rows=M // 2)
        o = (o[0] if isinstance(o, tuple) else o).float()
        first = _GEGLU_FIRST.setdefault(name, (o, pre.float().clone()))  # same seeded operands every variant
        name += f" d={(o - first[0]).abs().max().item():.1e}/{(pre.float() - first[1]).abs().max().item():.1e}"
        rows.append((name, f"{M}x{2 * F}x{Kd}", ms, 2 * M * 2 * F * Kd / ms / 1e9))
    for (M, F, Kd, name) in [(L2, 5120, 1280, "L2 geglu bwd"), (L1, 2560, 640, "L1 geglu bwd")]:
        dy = torch.randn(M, Kd, device=dev).bfloat16()
        wt = (torch.randn(F, Kd, device=dev) / Kd ** 0.5).bfloat16()  # ff.out weight transposed: [F, C]
        pre = torch.randn(M, 2 * F, device=dev).bfloat16()
        ms = t_ms(lambda: K.gemm_geglu_bwd(dy, wt, pre))
        rows.append((name, f"{M}x{F}x{Kd} +pre", ms, 2 * M * F * Kd / ms / 1e9))
    convs = [] if os.environ.get("GEMM_ONLY_GEGLU") else [(Bi, 128, 320, 320, "L0 conv 320", K.CONV_NORMAL),
                                       (Bi, 64, 640, 640, "L1 conv 640", K.CONV_NORMAL),
                                       (Bi, 32, 1280, 1280, "L2 conv 1280", K.CONV_NORMAL),
                                       (Bi, 32, 2560, 1280, "L2 conv 2560->1280", K.CONV_NORMAL),
                                       (Bi, 64, 1280, 1280, "up conv 1280 @64->128", K.CONV_UP2)]
    for (B, H, Ci, Co, name, mode) in convs:
        x = torch.randn(B, H, H, Ci, device=dev).bfloat16()
        w = torch.randn(Co, 3, 3, Ci, device=dev).bfloat16()
        Ho = 2 * H if mode == K.CONV_UP2 else H
        ms = t_ms(lambda: K.conv2d(x, w, mode=mode))
        rows.append((name, f"B{B} {H}^2 {Ci}->{Co}", ms, 2 * B * Ho * Ho * Co * 9 * Ci / ms / 1e9))
    for r in ([] if quiet else rows):
        print(f"{r[0]:24s} {r[1]:22s} {r[2]:8.3f} ms  {r[3]:7.1f} TFLOP/s")


if __name__ == "__main__":
    main()
