"""Same-process A/B of GEMM dispatch variants on the bs = 1 / GPU step (lora_bs1: 1 pair, gas 1) and optionally the
C5 DreamBooth micro-step shapes, alternating arms; CONFIG=c3 / c2 runs the bench's c3 object / the C2 headline instead.
usage (GPU): GEMM_VARIANTS=0,55 [CONFIG=c3] python tools/bs1_variant_ab.py [rounds]"""
import os
os.environ.setdefault("PSO_LIB", "knobs")  # benchmark knobs: the tools build (include/pso_amd_knobs.h)
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from pairwise_sample_optimization_amd import kernels as K  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    variants = [int(v) for v in os.environ.get("GEMM_VARIANTS", "0,55").split(",")]
    sys.argv = [sys.argv[0], "--no-cpu-baseline"]
    args = bench.parse()
    args.pairs, args.gas = 1, 1
    if os.environ.get("CONFIG") == "c3":  # the bench's c3 object: full-UNet DMD2, 4-step sampler
        args.full_unet, args.mode, args.num_steps = True, "dmd", 4
    elif os.environ.get("CONFIG") == "c2":
        args.pairs, args.gas = 2, 2
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    unet, tr, buf, g = bench.build(args, dev)
    imgs = 2 * args.pairs * args.gas * (args.num_steps - 1)
    res = {v: [] for v in variants}
    for r in range(rounds):
        for v in variants:
            K.gemm_set_variant(v)
            for _ in range(2):
                bench.one_step(tr, buf, g)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            n = 10 if os.environ.get("CONFIG") not in ("c3", "c2") else 4
            for _ in range(n):
                bench.one_step(tr, buf, g)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / n
            res[v].append(dt * 1e3)
            print(f"round {r} variant {v}: {dt * 1e3:.2f} ms/step  {imgs / dt:.2f} imgs/s", flush=True)
    K.gemm_set_variant(0)
    for v in variants:
        x = sorted(res[v])
        print(f"variant {v}: median {x[len(x) // 2]:.2f} ms/step", flush=True)


if __name__ == "__main__":
    main()
