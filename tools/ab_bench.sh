#!/bin/bash
# Same-box A/B of GEMM dispatch variants on the C2 bench step, interleaved: tools/ab_bench.sh "0 31" [rounds]
vars=${1:-"0 31"}; rounds=${2:-2}
for r in $(seq 1 $rounds); do
  for v in $vars; do
    out=$(PSO_BENCH_GEMM_VARIANT=$v timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline 2>/dev/null | tail -1) || exit $?
    echo "variant $v round $r: $(echo "$out" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "imgs/s", d["ms_per_step"], "ms")')"
  done
done
