"""Average kernel duration per (kernel, grid size) from a rocprofv3 kernel trace: the attention micro-benchmark runs
every variant on several shapes, and the per-name stats mix them.  usage: python tools/trace_by_grid.py DIR [filter]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    root = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else ""
    agg = defaultdict(list)
    for f in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                name = r["Kernel_Name"].replace("void ", "").split("(")[0]
                if pat not in name:
                    continue
                grid = int(r.get("Grid_Size", 0) or 0) or (int(r.get("Grid_Size_X", 0) or 0) * int(r.get("Grid_Size_Y", 1) or 1) *
                                                       int(r.get("Grid_Size_Z", 1) or 1))
                agg[(name, grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for (name, grid), v in sorted(agg.items()):
        v.sort()
        print(f"{name[:60]:60s} grid {grid:8d} n {len(v):4d} median {v[len(v) // 2]:9.1f} us  min {v[0]:9.1f} us")


if __name__ == "__main__":
    main()
