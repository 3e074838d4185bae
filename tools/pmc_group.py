"""HBM traffic of the 8-phase GEMMs per raster group (run under rocprofv3 --pmc FETCH_SIZE): for each group size,
REPS launches of each shape, in a fixed order, so the counter rows map back to (group, shape) by dispatch index.
Prints the launch plan; tools/parse_pmc_group.py joins it with the counter CSV."""
import os
os.environ.setdefault("PSO_LIB", "knobs")  # benchmark knobs: the tools build (include/pso_amd_knobs.h)
import sys
import json
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pairwise_sample_optimization_amd import kernels as K  # noqa: E402

SHAPES = [(16384, 1280, 1280), (16384, 1280, 5120), (65536, 640, 640), (65536, 640, 2560), (12288, 1280, 5120)]
GROUPS = [int(g) for g in os.environ.get("PMC_GROUPS", "1,2,4,8,16").split(",")]
REPS = 3


def main():
    dev = torch.device("cuda")
    ops = {s: (torch.randn(s[0], s[2], device=dev).bfloat16(), torch.randn(s[1], s[2], device=dev).bfloat16())
           for s in SHAPES}
    plan = []
    for g in GROUPS:
        K.gemm_set_variant(100 * g)  # g = 0: the automatic group (XCD-chunk aligned)
        for s in SHAPES:
            a, w = ops[s]
            for _ in range(REPS):
                K.gemm(a, w)
                plan.append({"group": g, "shape": s, "algo_bytes": 2 * (s[0] * s[2] + s[1] * s[2] + s[0] * s[1])})
    torch.cuda.synchronize()
    K.gemm_set_variant(0)
    print(json.dumps(plan))


if __name__ == "__main__":
    main()
