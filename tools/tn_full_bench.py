"""Full-weight TN GEMM (dW = X^T dY over the tokens, C3 / C4 full-UNet gradients) on the C3 step's shapes: TF/s of the
automatic dispatch under each GEMM variant (56 = the 256 x 256 TN tiles off), and the rel-L2 distance to torch fp32.
usage (GPU): python tools/tn_full_bench.py [variant ...]"""
import os
os.environ.setdefault("PSO_LIB", "knobs")  # benchmark knobs: the tools build (include/pso_amd_knobs.h)
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pairwise_sample_optimization_amd import kernels as K  # noqa: E402
from tools.gemm_bench import t_ms  # noqa: E402

SHAPES = [(6144, 10240, 1280, "geglu"), (6144, 1280, 1280, ""), (6144, 1280, 5120, ""), (6144, 3840, 1280, ""),
          (6144, 1280, 11520, ""), (24576, 1280, 11520, ""), (6144, 5120, 1280, ""), (24576, 5120, 640, "geglu"),
          (24576, 640, 640, "")]


def main():
    vs = [int(v) for v in sys.argv[1:]] or [0, 56]
    dev = torch.device("cuda")
    print("shape M x I x J      " + " ".join(f"{'v%d' % v:>14s}" for v in vs), flush=True)
    for (M, I, J, kind) in SHAPES:
        g = torch.Generator(device=dev).manual_seed(M + I + J)
        a = torch.randn(M, I, device=dev, generator=g).bfloat16()
        b = torch.randn(M, J, device=dev, generator=g).bfloat16()
        if kind == "geglu":  # a in the GEGLU interleave, the product in natural order
            ref = a.float()[:, torch.argsort(K.geglu_interleave_index(I // 2, dev))].T @ b.float()
        else:
            ref = a.float().T @ b.float()
        cells = []
        for v in vs:
            K.gemm_set_variant(v)
            out = torch.zeros(I, J, device=dev)
            fn = (lambda: K.gemm_tn_geglu(a, b, out)) if kind == "geglu" else (lambda: K.gemm_tn(a, b, out))
            fn()
            rel = ((out - ref).norm() / ref.norm()).item()
            ms = t_ms(fn, it=10)
            cells.append(f"{2.0 * M * I * J / ms / 1e9:6.0f} ({rel:.0e})")
        K.gemm_set_variant(0)
        print(f"{M:6d} x {I:5d} x {J:5d} {kind:5s} " + " ".join(f"{c:>14s}" for c in cells), flush=True)


if __name__ == "__main__":
    main()
