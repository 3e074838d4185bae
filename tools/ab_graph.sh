#!/bin/bash
# Same-box A/B of eager launches vs the hipGraph-captured epoch on the C2 step (each arm under its own time limit).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq 1 ${1:-2}); do
  for a in eager graph; do
    fl=""; [ $a = graph ] && fl="--graph"
    timeout -k 10 400 python -u bench.py --steps ${STEPS:-8} --warmup 3 --no-cpu-baseline --no-roofline $fl \
        > gpurun_out/ab_graph_$a.json 2> gpurun_out/ab_graph_$a.err || { tail -5 gpurun_out/ab_graph_$a.err; exit 1; }
    echo "$a round $r: $(python3 -c "import json;d=json.load(open('gpurun_out/ab_graph_$a.json'));print(d['value'],'imgs/s',d['ms_per_step'],'ms')")"
  done
done
