"""The bench's VAE decode object under a profiler: 8 latents 128x128 -> 8 images at 1024^2, one warm-up + DECODES timed
decodes (bench.vae_metric's workload without its own roofline pass).  Summarise a rocprofv3 kernel trace of it with
    python tools/vae_prof.py --summary TRACE_CSV DECODES+1
usage (GPU): rocprofv3 --kernel-trace --stats -d gpurun_out/vae_prof -o run -- python3 tools/vae_prof.py"""
import csv
import os
import sys
import time
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

DECODES = 3
TFLOP_PER_IMG = 10.49  # SURVEY §8a a7 (bench.VAE_DEC_TFLOP_PER_IMG)


def summary(path, ncalls):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    # main() idles 1 s after weight init / prepare: the decodes are the dispatches after the longest gap
    gaps = [int(rows[i + 1]["Start_Timestamp"]) - int(rows[i]["End_Timestamp"]) for i in range(len(rows) - 1)]
    rows = rows[gaps.index(max(gaps)) + 1:]
    per = defaultdict(lambda: [0, 0.0])
    t0, t1 = None, None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        per[r["Kernel_Name"].split("(")[0].replace("void ", "")][0] += 1
        per[r["Kernel_Name"].split("(")[0].replace("void ", "")][1] += (e - s) * 1e-3
        t0 = s if t0 is None else min(t0, s)
        t1 = e if t1 is None else max(t1, e)
    tot = sum(v[1] for v in per.values())
    fam = sum(v[1] for k, v in per.items() if k.startswith(("gemm", "(anonymous namespace)::gemm8p")))
    print(f"# per decode (trace total / {ncalls} decodes): kernel-busy {tot / ncalls / 1e3:.2f} ms, "
          f"{len(rows) / ncalls:.0f} dispatches; GEMM family {fam / ncalls / 1e3:.2f} ms")
    print(f"# 8 images x {TFLOP_PER_IMG} TF = {8 * TFLOP_PER_IMG:.1f} TF per decode -> "
          f"{8 * TFLOP_PER_IMG / (tot / ncalls * 1e-6):.0f} TF/s on kernel-busy time")
    print("| kernel | calls / decode | ms / decode | share | avg us |\n|---|---|---|---|---|")
    for k, (n, us) in sorted(per.items(), key=lambda x: -x[1][1])[:25]:
        print(f"| `{k[:90]}` | {n / ncalls:.0f} | {us / ncalls / 1e3:.3f} | {us / tot:.1%} | {us / n:.1f} |")


def main():
    import torch
    from pairwise_sample_optimization_amd.vae import AutoencoderKL, VAEConfig
    dev = torch.device("cuda")
    with torch.device(dev):
        vae = AutoencoderKL(VAEConfig())
    vae.init_weights(0)
    vae.prepare()
    g = torch.Generator(device=dev).manual_seed(7)
    lat = torch.randn(8, 128, 128, 4, device=dev, generator=g)
    torch.cuda.synchronize()
    time.sleep(1.0)  # marks the start of the decodes in a kernel trace (summary: after the longest idle gap)
    vae.decode_latents_nhwc(lat)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(DECODES):
        vae.decode_latents_nhwc(lat)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / DECODES
    print(f"vae decode: {ms:.2f} ms per 8-image decode ({8 * TFLOP_PER_IMG / ms * 1e3:.0f} TF/s)", flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--summary":
        summary(sys.argv[2], int(sys.argv[3]))
    else:
        main()
