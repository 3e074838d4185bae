"""Summarise a rocprofv3 kernel-trace (+ optional PMC FETCH_SIZE / WRITE_SIZE passes) of bench.py into
profiles/<tag>_*.  The GEMM family (gemm_bf16_kernel<...> + gemm_tn_kernel) average launch duration is taken over the
LAST `launches_per_step * steps` family launches of the trace (= the timed train steps, sampling excluded) so it is
comparable with bench.py's live HIP-event figure.

usage: python tools/parse_prof.py TAG [gpurun_out]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

FAMILY = ("gemm_bf16_kernel", "gemm_tn", "gemm_skinny")


def short(name):
    n = name.replace("void ", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0][:90]


def load_trace(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    rows.sort()
    return rows


def load_pmc(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        return None
    out = []
    with open(files[0]) as f:
        for r in csv.DictReader(f):
            out.append((int(r["Dispatch_Id"]), r["Kernel_Name"], r["Counter_Name"], float(r["Counter_Value"])))
    out.sort()
    return out


def main():
    tag = sys.argv[1]
    root = sys.argv[2] if len(sys.argv) > 2 else "gpurun_out"
    os.makedirs("profiles", exist_ok=True)
    bench = json.load(open(os.path.join(root, "bench.json")))
    rl = bench.get("roofline", {})
    steps_prof = 2
    trace = load_trace(glob.glob(os.path.join(root, "prof", "**", "*kernel_trace.csv"), recursive=True)[0])
    agg = defaultdict(lambda: [0, 0])
    for _, n, d in trace:
        agg[short(n)][0] += 1
        agg[short(n)][1] += d
    tot = sum(v[1] for v in agg.values())
    fam = [d for _, n, d in trace if any(f in n for f in FAMILY)]
    lps = rl.get("launches_per_step")
    timed = fam[-lps * steps_prof:] if lps else fam
    fam_avg_us = sum(timed) / max(len(timed), 1) / 1e3
    lines = [f"# {tag}: rocprofv3 --kernel-trace --stats of `python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline "
             f"--no-roofline` (C2 config, 1x MI355X)", "",
             f"Whole-run kernel time {tot / 1e9:.3f} s over {len(trace)} dispatches (incl. build + sampling).", "",
             "| kernel | calls | total ms | share | avg us |", "|---|---|---|---|---|"]
    for k, (c, d) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:40]:
        lines.append(f"| `{k}` | {c} | {d / 1e6:.1f} | {100 * d / tot:.2f}% | {d / c / 1e3:.1f} |")
    lines += ["", "## Dominant kernel family (roofline)", "",
              f"GEMM family launches in the 2 timed steps: {len(timed)} (bench: {lps} per step)",
              f"rocprof average launch duration: **{fam_avg_us:.2f} us**; bench.py live HIP-event average: "
              f"**{rl.get('avg_launch_us')} us** (events add ~1-3 us of record overhead per launch)."]
    traffic = None
    pf, pw = load_pmc(os.path.join(root, "pmc_fetch")), load_pmc(os.path.join(root, "pmc_write"))
    if pf and pw:
        def last_step(rows):
            fr = [(i, v) for i, n, c, v in rows if any(f in n for f in FAMILY)]
            return fr[-lps:] if lps else fr
        fs, ws = last_step(pf), last_step(pw)
        # FETCH_SIZE / WRITE_SIZE are in KiB; gfx950 FETCH_SIZE counts half the bytes of wide streaming reads
        fetch_b = 2 * 1024 * sum(v for _, v in fs) / max(len(fs), 1)
        write_b = 1024 * sum(v for _, v in ws) / max(len(ws), 1)
        traffic = fetch_b + write_b
        lines += ["", "## HBM traffic (PMC passes, one train step, GEMM family only)", "",
                  f"launches: fetch pass {len(fs)}, write pass {len(ws)}",
                  f"per launch: FETCH {fetch_b / 1e6:.2f} MB (FETCH_SIZE x 2, gfx950 correction) + WRITE "
                  f"{write_b / 1e6:.2f} MB = **{traffic / 1e6:.2f} MB**"]
        if rl.get("bytes_per_launch"):
            lines.append(f"algorithmic bytes per launch (A + B + C once): {rl['bytes_per_launch'] / 1e6:.2f} MB")
        json.dump({"traffic_bytes_per_launch": traffic, "fetch_bytes": fetch_b, "write_bytes": write_b,
                   "launches": len(fs), "source": f"profiles/{tag}_summary.md"},
                  open(f"profiles/{tag}_traffic.json", "w"), indent=1)
    lines += ["", "bench line of the same round:", "", "```", json.dumps(bench), "```"]
    open(f"profiles/{tag}_summary.md", "w").write("\n".join(lines) + "\n")
    stats = glob.glob(os.path.join(root, "prof", "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        with open(stats[0]) as f, open(f"profiles/{tag}_kernel_stats.csv", "w") as g:
            for i, line in enumerate(f):
                if i > 60:
                    break
                g.write(line)
    print("\n".join(lines[:60]))


if __name__ == "__main__":
    main()
