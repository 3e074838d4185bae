"""Join tools/pmc_group.py's launch plan with its rocprofv3 FETCH_SIZE counters: read bytes per launch vs the
algorithmic A + B and the A + 8 B model (every weight tile fetched once into each XCD's L2).
  usage: python3 tools/parse_pmc_group.py <plan.json> <run_counter_collection.csv>"""
import collections
import csv
import json
import re
import sys


def main(plan_path, csv_path):
    plan = json.load(open(plan_path))
    by = collections.OrderedDict()
    for r in csv.DictReader(open(csv_path)):
        by.setdefault(int(r["Dispatch_Id"]), []).append(r)
    disp = sorted(by)
    assert len(disp) == len(plan), (len(disp), len(plan))
    print("HBM read traffic of the 8-phase GEMM per raster group (tools/pmc_group.py under rocprofv3 --pmc FETCH_SIZE;")
    print("FETCH_SIZE x 2 gfx950 correction; group 0 = automatic); model = A + 8 B (each weight tile once per XCD L2)")
    print(f"{'M x N x K':>20} {'group':>5} {'fetch MB':>9} {'A+B MB':>8} {'ratio':>6} {'A+8B MB':>8}  kernel")
    agg = collections.defaultdict(list)
    for d, p in zip(disp, plan):
        fetch = sum(float(r["Counter_Value"]) for r in by[d]) * 2 * 1024
        m = re.search(r"gemm\w*<[^>]*>", by[d][0]["Kernel_Name"])
        agg[(tuple(p["shape"]), p["group"])].append((fetch, m.group(0) if m else by[d][0]["Kernel_Name"][:50]))
    for (s, g), v in sorted(agg.items()):
        M, N, Kd = s
        A, B = 2 * M * Kd, 2 * N * Kd
        f = sum(x[0] for x in v) / len(v)
        print(f"{M:>6} x {N:>5} x {Kd:>5} {g:>5} {f / 1e6:9.1f} {(A + B) / 1e6:8.1f} {f / (A + B):6.2f} "
              f"{(A + 8 * B) / 1e6:8.1f}  {v[0][1]}")


if __name__ == "__main__":
    main(*sys.argv[1:3])
