"""Per-kernel breakdown of the steady-state window of a rocprofv3 kernel trace, delimited by a marker kernel that runs
once per step (e.g. db_finalize_kernel for the DreamBooth micro-step): from the `skip`-th marker to the last one.
usage: python tools/window_breakdown.py TRACE_CSV MARKER [skip] [top]"""
import csv
import sys
from collections import defaultdict


def main():
    path, marker = sys.argv[1], sys.argv[2]
    skip = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    top = int(sys.argv[4]) if len(sys.argv) > 4 else 30
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(path)))
    idx = [i for i, r in enumerate(rows) if r[2].startswith(marker)]
    k0, k1 = idx[skip], idx[-1]
    n = len(idx) - 1 - skip
    win = rows[k0 + 1:k1 + 1]
    agg = defaultdict(lambda: [0, 0])
    for s, e, nm in win:
        k = nm.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:80]
        agg[k][0] += 1
        agg[k][1] += e - s
    busy = sum(v[1] for v in agg.values())
    print(f"window {n} steps: {len(win) / n:.0f} dispatches/step, wall {(win[-1][1] - win[0][0]) / 1e6 / n:.2f} ms/step, "
          f"kernel-busy {busy / 1e6 / n:.2f} ms/step")
    for k, (c, d) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{d / 1e6 / n:7.2f} ms/step {100 * d / busy:5.1f}%  n/step={c / n:5.0f}  avg {d / c / 1e3:7.1f} us  {k}")


if __name__ == "__main__":
    main()
