"""Micro-benchmark of the flash-attention kernels on the SDXL UNet shapes (8 images at 1024^2).
usage: ATTN_VARIANTS=0,22,44 (fwd + 10*bwd + 10000*nb of the short-KV forward, 990000 = its one-block form)
       ATTN_IMAGES=16 python tools/attn_bench.py   (GPU)"""
import hashlib
import os
os.environ.setdefault("PSO_LIB", "knobs")  # benchmark knobs: the tools build (include/pso_amd_knobs.h)
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pairwise_sample_optimization_amd import kernels as K  # noqa: E402


def t_ms(fn, it=10):
    for _ in range(2):
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
    Bi = int(os.environ.get("ATTN_IMAGES", "8"))
    shapes = [("L1 self", Bi, 10, 4096, 4096), ("L2 self", Bi, 20, 1024, 1024), ("L1 cross", Bi, 10, 4096, 77),
              ("L2 cross", Bi, 20, 1024, 77)]
    if os.environ.get("ATTN_CROSS_ONLY"):
        shapes = [x for x in shapes if x[4] <= 128]
    if os.environ.get("ATTN_SHAPE"):  # one level only, e.g. "L2 cross"
        shapes = [x for x in shapes if x[0] == os.environ["ATTN_SHAPE"]]
    ref = {}
    for v in [int(x) for x in os.environ.get("ATTN_VARIANTS", "0").split(",")]:
        K.lib().pso_attention_set_variant(v)
        print(f"--- variant {v} ---")
        for name, B, H, Sq, Sk in shapes:
            C = H * 64
            torch.manual_seed(Sq * 7 + Sk)
            q = torch.randn(B, Sq, 3 * C, device=dev).bfloat16()[..., :C]
            k = torch.randn(B, Sk, C, device=dev).bfloat16()
            vv = torch.randn(B, Sk, C, device=dev).bfloat16()
            fl = 4 * B * H * Sq * Sk * 64
            ms = t_ms(lambda: K.attention_fwd(q, k, vv, H))
            o, lse = K.attention_fwd(q, k, vv, H)
            do = torch.randn(B, Sq, C, device=dev).bfloat16()
            msb = t_ms(lambda: K.attention_bwd(q, k, vv, o, lse, do, H))
            grads = K.attention_bwd(q, k, vv, o, lse, do, H)
            outs = (o, lse, *grads)
            same = ""
            if name in ref:  # every variant must give the bits of the first one (same arithmetic, other schedule)
                same = " bits " + ("identical" if all(torch.equal(x, y) for x, y in zip(outs, ref[name])) else
                                   "DIFFER (max %.3g)" % max((x.float() - y.float()).abs().max().item()
                                                            for x, y in zip(outs, ref[name])))
            else:
                ref[name] = [x.clone() for x in outs]
            # digest of the outputs: compares builds of the same sources (same-box library A/B via PSO_LIB_PATH)
            dig = hashlib.sha1(b"".join(x.view(torch.int16).cpu().numpy().tobytes() for x in (o, *grads))).hexdigest()
            print(f"{name:10s} B{B} H{H} {Sq}x{Sk}: fwd {ms:7.3f} ms {fl / ms / 1e9:7.1f} TF/s | "
                  f"bwd {msb:7.3f} ms {2.5 * fl / msb / 1e9:7.1f} TF/s (2.5x fwd flop){same} sha1 {dig[:12]}", flush=True)
    K.lib().pso_attention_set_variant(0)


if __name__ == "__main__":
    main()
