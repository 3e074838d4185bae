"""Per-kernel breakdown of the TIMED train steps inside a rocprofv3 kernel trace of bench.py.
The window runs from the end of the optimizer launch that closed the last warmup step to the end of the last step's
optimizer launch (one AdamW launch per step); without steps + 1 of them, from the first GEMM-family dispatch of the
last `steps * launches_per_step` family dispatches.
usage: python tools/step_breakdown.py TRACE_CSV LAUNCHES_PER_STEP STEPS"""
import csv
import sys
from collections import defaultdict

FAMILY = ("gemm_bf16_kernel", "gemm8p_kernel", "gemm_tn", "gemm_skinny")


def short(name):
    n = name.replace("void ", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0][:80]


def main():
    path, lps, steps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    opt = [i for i, r in enumerate(rows) if "adamw" in r[2]]
    if len(opt) >= steps + 1:
        win = rows[opt[-steps - 1] + 1:opt[-1] + 1]
    else:
        fam = [i for i, r in enumerate(rows) if any(k in r[2] for k in FAMILY)]
        win = rows[fam[-lps * steps]:]
    t0, t1 = win[0][0], max(r[1] for r in win)
    agg = defaultdict(lambda: [0, 0])
    for s, e, n in win:
        agg[short(n)][0] += 1
        agg[short(n)][1] += e - s
    busy = sum(v[1] for v in agg.values())
    print(f"window {len(win)} dispatches, wall {(t1 - t0) / 1e6 / steps:.2f} ms/step, kernel-busy "
          f"{busy / 1e6 / steps:.2f} ms/step")
    for k, (c, d) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:45]:
        print(f"{d / 1e6 / steps:8.2f} ms/step {100 * d / busy:5.1f}%  n/step={c / steps:6.0f}  avg {d / c / 1e3:7.1f} us  {k}")


if __name__ == "__main__":
    main()
