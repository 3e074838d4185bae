"""Segment timing of the ping-pong dK/dV kernel (attn_bwd_dkv_pp_kernel, TR form): workgroup 0's waves 0 and 4 record
the shader clock before and after every barrier; this prints, per group, the median work and barrier-wait time of its
A (matrix) and B (vector) segments.  The s_memtime stamps themselves add ~15 % to the kernel.
usage (GPU): PP_VARIANTS=1080,1090 python tools/pp_trace.py   (1000s digit: trace; 8x / 9x: the ping-pong form,
9x with raised A-segment priority -- see pso_attention_set_variant)"""
import ctypes
import os
os.environ.setdefault("PSO_LIB", "knobs")  # benchmark knobs: the tools build (include/pso_amd_knobs.h)
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pairwise_sample_optimization_amd import kernels as K  # noqa: E402


def report(L):
    buf = (ctypes.c_ulonglong * 1040)()
    assert L.pso_attn_pp_trace(buf) == 0
    t = [list(buf[:520]), list(buf[520:])]
    med = lambda x: sorted(x)[len(x) // 2]
    for gi in range(2):
        # stamps: [end of work, segment start] per segment: t[2j] = end of work of the previous segment, t[2j+1] = start
        # of segment j (A, B alternating from j = 0)
        st = t[gi][1::2][:120]
        en = t[gi][2::2][:120]
        work = [en[j] - st[j] for j in range(100)]
        wait = [st[j + 1] - en[j] for j in range(100)]
        print(f"  group {gi}: A work {med(work[4::2])} wait {med(wait[4::2])} | B work {med(work[5::2])} "
              f"wait {med(wait[5::2])}", flush=True)


def main():
    L = K.lib()
    dev = torch.device("cuda")
    B, H, S = 8, 10, 4096
    C = H * 64
    torch.manual_seed(0)
    q, k, v = (torch.randn(B, S, C, device=dev).bfloat16() for _ in range(3))
    o, lse = K.attention_fwd(q, k, v, H)
    do = torch.randn(B, S, C, device=dev).bfloat16()
    for var in [int(x) for x in os.environ.get("PP_VARIANTS", "1080").split(",")]:
        L.pso_attention_set_variant(var)
        for _ in range(3):
            K.attention_bwd(q, k, v, o, lse, do, H)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            K.attention_bwd(q, k, v, o, lse, do, H)
        e1.record()
        torch.cuda.synchronize()
        print(f"variant {var}: bwd {e0.elapsed_time(e1) / 5:.3f} ms", flush=True)
        report(L)
    L.pso_attention_set_variant(0)


if __name__ == "__main__":
    main()
