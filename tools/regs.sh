#!/bin/bash
# Register / scratch / occupancy table of every kernel in one .hip file: tools/regs.sh <file.hip> [name-filter]
f=$1; pat=${2:-.}
cd "$(dirname "$0")/../pairwise_sample_optimization_amd/csrc" || exit 1
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -munsafe-fp-atomics -c "$f" -o /tmp/regs_probe.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c '
import re, sys
rows, cur = [], None
for line in sys.stdin:
    m = re.search(r"remark:\s+(Function Name|VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]): (\S+)", line)
    if not m: continue
    k, v = m.groups()
    if k == "Function Name": cur = {"name": v}; rows.append(cur)
    else: cur[k.split()[0]] = v
for r in rows:
    if re.search(sys.argv[1], r["name"]):
        print("%4s %4s scr=%5s occ=%s %s" % (r.get("VGPRs"), r.get("AGPRs"), r.get("ScratchSize"), r.get("Occupancy"), r["name"][:110]))
' "$pat"
