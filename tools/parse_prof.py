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

FAMILY = ("gemm_bf16_kernel", "gemm8p_kernel", "gemm_tn", "gemm_skinny")


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
    dom = rl.get("kernel", "")
    lps = rl.get("launches_per_step")
    mine = [d for _, n, d in trace if short(n).startswith(dom)] if dom else []
    timed = mine[-lps * steps_prof:] if lps else mine
    dom_avg_us = sum(timed) / max(len(timed), 1) / 1e3
    fam = [d for _, n, d in trace if any(f in n for f in FAMILY)]
    flps = rl.get("family", {}).get("launches_per_step")
    ftimed = fam[-flps * steps_prof:] if flps else fam
    lines = [f"# {tag}: rocprofv3 --kernel-trace --stats of `python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline "
             f"--no-roofline` (C2 config, 1x MI355X)", "",
             f"Whole-run kernel time {tot / 1e9:.3f} s over {len(trace)} dispatches (incl. build + sampling).", "",
             "| kernel | calls | total ms | share | avg us |", "|---|---|---|---|---|"]
    for k, (c, d) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:40]:
        lines.append(f"| `{k}` | {c} | {d / 1e6:.1f} | {100 * d / tot:.2f}% | {d / c / 1e3:.1f} |")
    lines += ["", "## Dominant kernel (roofline)", "",
              f"kernel `{dom}`: {len(timed)} launches in the 2 timed steps (bench: {lps} per step)",
              f"rocprof average launch duration: **{dom_avg_us:.2f} us**; bench.py live HIP-event average: "
              f"**{rl.get('avg_launch_us')} us** (an event pair adds ~1-3 us per launch).",
              f"algorithmic flop per launch {rl.get('flop_per_launch', 0) / 1e9:.2f} GF -> "
              f"{rl.get('flop_per_launch', 0) / (dom_avg_us * 1e-6) / 1e12 if dom_avg_us else 0:.1f} TF/s on the "
              f"rocprof duration (bench: {rl.get('achieved')} TF/s)", "",
              f"GEMM family: {len(ftimed)} launches in the timed steps, rocprof average "
              f"{sum(ftimed) / max(len(ftimed), 1) / 1e3:.2f} us (bench {rl.get('family', {}).get('achieved')} TF/s)"]
    traffic = None
    pf, pw = load_pmc(os.path.join(root, "pmc_fetch")), load_pmc(os.path.join(root, "pmc_write"))
    if pf and pw and dom:
        def last_step(rows):
            fr = [(i, v) for i, n, c, v in rows if short(n).startswith(dom)]
            return fr[-lps:] if lps else fr
        fs, ws = last_step(pf), last_step(pw)
        # FETCH_SIZE / WRITE_SIZE are in KiB; gfx950 FETCH_SIZE counts half the bytes of wide streaming reads
        fetch_b = 2 * 1024 * sum(v for _, v in fs) / max(len(fs), 1)
        write_b = 1024 * sum(v for _, v in ws) / max(len(ws), 1)
        traffic = fetch_b + write_b
        lines += ["", f"## HBM traffic of `{dom}` (PMC passes, one train step)", "",
                  f"launches: fetch pass {len(fs)}, write pass {len(ws)}",
                  f"per launch: FETCH {fetch_b / 1e6:.2f} MB (FETCH_SIZE x 2, gfx950 correction) + WRITE "
                  f"{write_b / 1e6:.2f} MB = **{traffic / 1e6:.2f} MB**"]
        if rl.get("bytes_per_launch"):
            lines.append(f"algorithmic bytes per launch (A + B + C once): {rl['bytes_per_launch'] / 1e6:.2f} MB "
                         f"(ratio {traffic / rl['bytes_per_launch']:.2f})")
        json.dump({"kernel": dom, "src_hash": rl.get("src_hash"), "traffic_bytes_per_launch": traffic,
                   "fetch_bytes": fetch_b, "write_bytes": write_b, "launches": len(fs),
                   "source": f"profiles/{tag}_summary.md"}, open(f"profiles/{tag}_traffic.json", "w"), indent=1)
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
