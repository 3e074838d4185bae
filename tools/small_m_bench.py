"""GEMM tile variants on the shapes of the bs = 1 / GPU step (1 pair: 2 policy + 2 reference images per paired pass;
the backward runs on the 2 policy images): every variant of pso_gemm_set_variant given in GEMM_VARIANTS, per shape,
with the LoRA K-tail where the step has one, next to hipBLASLt (torch.mm) on the same operands.
usage (GPU): GEMM_VARIANTS=0,3,6,12,20,21,22 python tools/small_m_bench.py"""
import os
os.environ.setdefault("PSO_LIB", "knobs")  # benchmark knobs: the tools build (include/pso_amd_knobs.h)
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pairwise_sample_optimization_amd import kernels as K  # noqa: E402

C3_SHAPES = [  # the full-UNet step at 6 images (BASELINE C3): L2 M = 6144, L1 M = 24576, no LoRA tail
    (6144, 1280, 1280, 0, 0), (6144, 1280, 5120, 0, 0), (6144, 3840, 1280, 0, 0), (6144, 1280, 10240, 0, 0),
    (6144, 5120, 1280, 0, 0), (24576, 640, 640, 0, 0), (24576, 640, 2560, 0, 0), (24576, 1920, 640, 0, 0),
    (24576, 640, 5120, 0, 0), (12288, 1280, 1280, 0, 0), (12288, 1280, 5120, 0, 0),
]
SHAPES = [  # (M, N, K, K2 LoRA tail, tail_rows)  from gpurun_out/shp.log (bs = 1)
    (2048, 1280, 10240, 0, 0), (2048, 1280, 1280, 32, 0), (2048, 1280, 3840, 96, 0), (4096, 1280, 1280, 32, 2048),
    (4096, 1280, 5120, 0, 0), (4096, 3840, 1280, 32, 2048), (8192, 640, 5120, 0, 0), (16384, 640, 640, 32, 8192),
    (8192, 640, 640, 32, 0), (4096, 1280, 1280, 0, 0), (2048, 1280, 1280, 0, 0), (8192, 640, 1920, 96, 0),
]


def t_ms(fn, it=30):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it


def geglu_bwd(dev, variants):
    """The fused GEGLU backward GEMM (dout = dy W_out^T, interleaved input gradient from the saved pre-activation) on
    the bs = 1 / C2 / C3 shapes."""
    print("geglu_bwd".ljust(34) + "".join(f"{'v' + str(v):>9}" for v in variants))
    for M, F, Kd in [(2048, 5120, 1280), (8192, 2560, 640), (8192, 5120, 1280), (32768, 2560, 640), (6144, 5120, 1280),
                     (24576, 2560, 640)]:
        dy = torch.randn(M, Kd, device=dev).bfloat16()
        wt = (torch.randn(F, Kd, device=dev) / Kd ** 0.5).bfloat16()
        pre = torch.randn(M, 2 * F, device=dev).bfloat16()
        line = f"{M}x{F}x{Kd}".ljust(34)
        for v in variants:
            K.gemm_set_variant(v)
            ms = t_ms(lambda: K.gemm_geglu_bwd(dy, wt, pre))
            line += f"{2 * M * F * Kd / ms / 1e9:8.0f} "
        K.gemm_set_variant(0)
        print(line, flush=True)


def skinny(dev):
    """The rank-r LoRA products (N = r): us per launch back to back, for the skinny kernel form in PSO_SKINNY_VARIANT
    (read once per process)."""
    print(f"skinny (PSO_SKINNY_VARIANT={os.environ.get('PSO_SKINNY_VARIANT', '0')})   us/launch   GB/s of A")
    for M, N, Kd in [(2048, 32, 1280), (2048, 96, 1280), (4096, 32, 1280), (8192, 32, 640), (2048, 32, 5120),
                     (8192, 32, 1280), (32768, 32, 640)]:
        a = torch.randn(M, Kd, device=dev).bfloat16()
        w = (torch.randn(N, Kd, device=dev) / Kd ** 0.5).bfloat16()
        out = K.gemm(a, w)
        ref = a.float() @ w.float().t()
        err = ((out.float() - ref).norm() / ref.norm()).item()
        us = 1e3 * t_ms(lambda: K.gemm(a, w), it=200)
        print(f"{M}x{N}x{Kd}".ljust(20) + f"{us:9.2f} {M * Kd * 2 / us / 1e3:9.0f}  err {err:.1e}  "
              f"{K.lib().pso_last_kernel().decode()}", flush=True)


def main():
    dev = torch.device("cuda")
    if os.environ.get("SKINNY"):
        return skinny(dev)
    if os.environ.get("GEGLU_BWD"):
        variants = [int(v) for v in os.environ.get("GEMM_VARIANTS", "0,0,31,45").split(",")]
        return geglu_bwd(dev, variants)
    x = torch.randn(8192, 8192, device=dev).bfloat16()
    for _ in range(200):
        x @ x
    torch.cuda.synchronize()
    torch.manual_seed(0)
    ops = []
    for M, N, Kd, K2, tr in (C3_SHAPES if os.environ.get("GEMM_C3") else SHAPES):
        a = torch.randn(M, Kd, device=dev).bfloat16()
        w = (torch.randn(N, Kd, device=dev) / Kd ** 0.5).bfloat16()
        kw = {}
        if K2:
            rows = tr if tr else M
            kw = dict(a2=torch.randn(rows, K2, device=dev).bfloat16(),
                      w2=(torch.randn(N, K2, device=dev) * 0.01).bfloat16(), tail_rows=tr)
        ref = a.float() @ w.float().t()
        if K2:
            ref[:kw["a2"].shape[0]] += kw["a2"].float() @ kw["w2"].float().t()
        ops.append(((M, N, Kd, K2, tr), a, w, kw, ref))
    variants = [int(v) for v in os.environ.get("GEMM_VARIANTS", "0,3,6,12,20,21,22").split(",")]
    print("shape".ljust(34) + "".join(f"{'v' + str(v):>9}" for v in variants) + "   hipBLASLt  (TF/s)")
    for key, a, w, kw, ref in ops:
        M, N, Kd, K2, tr = key
        fl = 2.0 * M * N * Kd + (2.0 * (tr or M) * N * K2 if K2 else 0)
        line = f"{M}x{N}x{Kd}+{K2}/{tr}".ljust(34)
        for v in variants:
            K.gemm_set_variant(v)
            try:
                out = K.gemm(a, w, **kw)
                err = ((out.float() - ref).norm() / ref.norm()).item()
                ms = t_ms(lambda: K.gemm(a, w, **kw))
                line += f"{fl / ms / 1e9:8.0f}{'!' if err > 1e-2 else ' '}"
            except Exception as e:  # variant not applicable to the shape
                line += f"{'-':>8} "
        K.gemm_set_variant(0)
        K.gemm(a, w, **kw)
        kname = K.lib().pso_last_kernel().decode().replace("gemm_bf16_kernel", "2p").replace("gemm8p_kernel", "8p")
        wt = w.t()
        line += f"{fl / t_ms(lambda: torch.mm(a, wt)) / 1e9:10.0f}   v0: {kname}"
        print(line, flush=True)


if __name__ == "__main__":
    main()
