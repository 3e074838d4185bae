"""Summarise tools/attn_pmc.sh (three rocprofv3 --pmc passes over tools/attn_bench.py) into a markdown table: per
attention kernel x grid size, counter averages per dispatch and the derived issue shares.
usage: python tools/parse_attn_pmc.py [gpurun_out/attn_pmc] > profiles/<tag>_attention_pmc.md"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(d):
    """(kernel, grid) -> counter -> list of per-dispatch values (summed over the dispatch's rows)."""
    out = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        per = defaultdict(float)
        key = {}
        with open(f) as fh:
            for r in csv.DictReader(fh):
                did = int(r["Dispatch_Id"])
                per[(did, r["Counter_Name"])] += float(r["Counter_Value"])
                name = r["Kernel_Name"].replace("void ", "").split("(")[0]
                key[did] = (name, int(r.get("Grid_Size", 0) or 0))
        for (did, cn), v in per.items():
            out[key[did]][cn].append(v)
    return out


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/attn_pmc"
    agg = defaultdict(dict)
    for p in sorted(glob.glob(os.path.join(root, "p*"))):
        if not os.path.isdir(p):
            continue
        for k, cs in load(p).items():
            for cn, vs in cs.items():
                agg[k][cn] = sum(vs) / len(vs)
    print("| kernel | grid | MFMA | VALU | TRANS | VALU/MFMA | MFMA busy | issue-stall | wait | LDS conflict/LDS active | LDS wait |")
    print("|---|---|---|---|---|---|---|---|---|---|---|")
    for (name, grid), c in sorted(agg.items()):
        if "attn" not in name or "SQ_INSTS_MFMA" not in c:
            continue
        mf, va, tr = c.get("SQ_INSTS_MFMA", 0), c.get("SQ_INSTS_VALU", 0), c.get("SQ_INSTS_VALU_TRANS_F32", 0)
        busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / 1024 / max(c.get("GRBM_GUI_ACTIVE", 1) / 8, 1)
        wc = max(c.get("SQ_WAVE_CYCLES", 1), 1)
        print(f"| `{name}` | {grid} | {mf / 1e6:.1f}M | {va / 1e6:.1f}M | {tr / 1e6:.1f}M | {va / max(mf, 1):.2f} | "
              f"{busy:.2f} | {c.get('SQ_WAIT_INST_ANY', 0) / wc:.2f} | {c.get('SQ_WAIT_ANY', 0) / wc:.2f} | "
              f"{c.get('SQ_LDS_BANK_CONFLICT', 0) / max(c.get('SQ_ACTIVE_INST_LDS', 1), 1):.2f} | "
              f"{c.get('SQ_WAIT_INST_LDS', 0) / wc:.2f} |")


if __name__ == "__main__":
    main()
