#!/bin/bash
# Same-box A/B of the C2 train step, interleaved rounds (every arm under its own time limit; stops at the first failure).
#   tools/ab.sh vars "0 31" [rounds]   GEMM dispatch variants (variant + 100 * raster group rows)
#   tools/ab.sh attn "0 100" [rounds]  attention variants
#   tools/ab.sh tree [rounds]          ab/prev (a snapshot of the previous commit with its built library) vs this tree
#   tools/ab.sh env "A=1 A=2,B=3" [rounds]   arbitrary environment settings per arm (comma-separated assignments)
# AB_ARGS adds bench.py arguments to every arm (e.g. the C3 full-UNet step), STEPS the timed steps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
kind=$1; shift
if [ "$kind" = tree ]; then arms="prev cur"; rounds=${1:-2}; else arms=${1:-"0"}; rounds=${2:-2}; fi
for r in $(seq 1 $rounds); do
  for a in $arms; do
    D=$PWD; envs=""
    case $kind in
      vars) envs="PSO_BENCH_GEMM_VARIANT=$a" ;;
      attn) envs="PSO_BENCH_ATTN_VARIANT=$a" ;;
      env) envs="${a//,/ }" ;;
      tree) [ $a = prev ] && D=$PWD/ab/prev ;;
    esac
    (cd $D && env $envs timeout -k 10 400 python -u bench.py --steps ${STEPS:-8} --warmup 3 --no-cpu-baseline --no-roofline --no-extra --epochs 0 ${AB_ARGS:-}) \
        > "gpurun_out/ab_${kind}_$a.json" 2> "gpurun_out/ab_${kind}_$a.err" || { tail -5 "gpurun_out/ab_${kind}_$a.err"; exit 1; }
    echo "$kind $a round $r: $(python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(d['value'],'imgs/s',d['ms_per_step'],'ms')" "gpurun_out/ab_${kind}_$a.json")"
  done
done
