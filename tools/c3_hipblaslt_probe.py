"""Probe (tools only, never the product path): the C3 full-UNet step with its plain bf16 products (no bias / residual /
LoRA tail / row bias / f32 accumulate -- the backward's input-gradient GEMMs) routed to hipBLASLt through torch.mm,
to size what a library GEMM would buy there.  usage (GPU): PROBE_LIB=1 python tools/c3_hipblaslt_probe.py <bench args>"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pairwise_sample_optimization_amd import kernels as K  # noqa: E402

_gemm = K.gemm
N_LIB = [0]


def gemm(a, w, *, bias=None, resid=None, a2=None, w2=None, alpha=1.0, rowbias=None, rows_per_group=1, out=None,
         out_dtype=K.BF16, accumulate=False, tail_group_n=0, tail_rows=0):
    plain = (bias is None and resid is None and a2 is None and rowbias is None and alpha == 1.0 and out is None and
             out_dtype == K.BF16 and not accumulate and a.shape[0] >= 2048)
    if plain and os.environ.get("PROBE_LIB") == "1":
        N_LIB[0] += 1
        return torch.mm(a, w.t())
    return _gemm(a, w, bias=bias, resid=resid, a2=a2, w2=w2, alpha=alpha, rowbias=rowbias,
                 rows_per_group=rows_per_group, out=out, out_dtype=out_dtype, accumulate=accumulate,
                 tail_group_n=tail_group_n, tail_rows=tail_rows)


K.gemm = gemm
import bench  # noqa: E402

if __name__ == "__main__":
    sys.argv = [sys.argv[0]] + sys.argv[1:]
    bench.main()
    print(f"[probe] plain products routed to torch.mm: {N_LIB[0]}", file=sys.stderr)
