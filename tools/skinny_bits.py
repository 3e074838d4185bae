"""Skinny-GEMM dispatch forms: a digest of the outputs and the per-launch time for the LoRA-down shapes (N <= 96) the
step runs, so two processes under different PSO_SKINNY_VARIANT values can be compared bit for bit.
usage (GPU): PSO_SKINNY_VARIANT=4 python tools/skinny_bits.py; python tools/skinny_bits.py   (compare the digests)"""
import hashlib
import os
os.environ.setdefault("PSO_LIB", "knobs")  # benchmark knobs: the tools build (include/pso_amd_knobs.h)
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pairwise_sample_optimization_amd import kernels as K  # noqa: E402

SHAPES = [(2048, 32, 1280, 1), (8192, 32, 1280, 1), (16384, 32, 1280, 1), (4096, 16, 1280, 1), (2048, 32, 1032, 1),
          (8192, 32, 640, 1), (2048, 32, 1280, 3), (8192, 32, 1280, 3), (1000, 32, 1280, 1),
          (2048, 96, 1280, 1), (4096, 96, 1280, 1), (2048, 64, 1280, 1)]


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    print(f"PSO_SKINNY_VARIANT={os.environ.get('PSO_SKINNY_VARIANT', '0')}", flush=True)
    for M, N, Kd, groups in SHAPES:
        a = torch.randn(M, Kd * groups, device=dev, generator=g).bfloat16()
        w = torch.randn(N, Kd * groups, device=dev, generator=g).bfloat16()
        f = (lambda: K.gemm(a, w)) if groups == 1 else (lambda: K.gemm_grouped_skinny(a, w, groups))
        out = f()
        torch.cuda.synchronize()
        dig = hashlib.sha1(out.view(torch.int16).cpu().numpy().tobytes()).hexdigest()[:16]
        for _ in range(20):
            f()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(200):
            f()
        e1.record()
        torch.cuda.synchronize()
        print(f"M={M} N={N} K={Kd} groups={groups}: {e0.elapsed_time(e1) / 200 * 1e3:.2f} us  digest {dig}",
              flush=True)


if __name__ == "__main__":
    main()
