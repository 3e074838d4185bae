"""8-bit AdamW (bitsandbytes AdamW8bit restated, optim.hip) over a C3-sized flat parameter buffer: ms per step and the
HBM rate on its 18 B per parameter (fp32 param read + write, fp32 grad read, two uint8 codes read + write, the bf16
working copy written).  Round 4: 11.8 ms over 2.567e9 parameters (3.9 TB/s); a persistent form (4 / 6 / 8
workgroups per CU walking the blocks, the maps loaded once per workgroup) ran 14.7 / 13.8 / 13.5 ms; 2 / 4 blocks per
workgroup 12.1 / 12.4 vs 11.9 ms; the contiguous element layout (PSO_ADAM8_LAYOUT=1, now the default) 11.44 / 11.50
vs 11.88 / 11.96 ms on one box, same bits; byte-offset search 10.86, branch-free non-finite skip 10.50 ms.
usage (GPU): python tools/adam8_bench.py [n_params]"""
import os
os.environ.setdefault("PSO_LIB", "knobs")  # benchmark knobs: the tools build (include/pso_amd_knobs.h)
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pairwise_sample_optimization_amd import kernels as K  # noqa: E402


def main():
    n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 2_567_000_000
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    p = torch.randn(n, device=dev, generator=g) * 0.02
    gr = torch.randn(n, device=dev, generator=g) * 1e-3
    pw = torch.empty(n, device=dev, dtype=torch.bfloat16)
    st = K.Adam8State(n, dev)
    for s in range(1, 3):
        K.adamw8bit_step(p, gr, st, 1e-5, (0.9, 0.999), 1e-8, 1e-2, s, out_bf16=pw)
    torch.cuda.synchronize()
    steps = 5
    t0 = time.perf_counter()
    for s in range(3, 3 + steps):
        K.adamw8bit_step(p, gr, st, 1e-5, (0.9, 0.999), 1e-8, 1e-2, s, out_bf16=pw)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    print(f"n={n:.3e}  {ms:.2f} ms/step  {18.0 * n / ms / 1e6:.0f} GB/s  checksum {p[:1 << 20].double().sum().item():.9e} "
          f"{st.qm[:1 << 20].double().sum().item():.0f}", flush=True)


if __name__ == "__main__":
    main()
