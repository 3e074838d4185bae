"""Per-shape breakdown of the GEMM family inside one C2 train step (HIP events per launch, grouped by shape).
usage: python tools/shape_prof.py [--top 40]  (GPU)"""
import os
os.environ.setdefault("PSO_LIB", "knobs")  # benchmark knobs: the tools build (include/pso_amd_knobs.h)
import sys
from collections import defaultdict

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from pairwise_sample_optimization_amd import kernels as K  # noqa: E402


def main():
    sys.argv = [sys.argv[0], "--no-cpu-baseline"] + sys.argv[1:]
    args = bench.parse()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    if os.environ.get("PSO_BENCH_GEMM_VARIANT"):
        K.gemm_set_variant(int(os.environ["PSO_BENCH_GEMM_VARIANT"]))
    unet, tr, buf, g = bench.build(args, dev)
    bench.one_step(tr, buf, g)
    torch.cuda.synchronize()
    K.PROFILE = []
    K.SideStream.enabled_any = False  # serial launches so every event pair times one kernel
    bench.one_step(tr, buf, g)
    torch.cuda.synchronize()
    rec, K.PROFILE = K.PROFILE, None
    agg = defaultdict(lambda: [0, 0.0, 0.0])
    kn = defaultdict(set)
    for fl, nb, e0, e1, tag, kname in rec:
        a = agg[tag]
        a[0] += 1
        a[1] += e0.elapsed_time(e1)
        a[2] += fl
        kn[tag].add(kname.replace("gemm8p_kernel", "8p").replace("gemm_bf16_kernel", "2p"))
    tot = sum(a[1] for a in agg.values())
    print(f"GEMM family: {len(rec)} launches, {tot:.1f} ms, {sum(a[2] for a in agg.values()) / tot / 1e9:.1f} TF/s")
    top = int(os.environ.get("SHAPE_TOP", "60"))
    for tag, (n, ms, fl) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{ms:8.2f} ms {100 * ms / tot:5.1f}% n={n:4d} {fl / ms / 1e9:7.1f} TF/s  {tag}  {'/'.join(sorted(kn[tag]))}")


if __name__ == "__main__":
    main()
