#!/bin/bash
# Profile the C2 step on the GPU box: rocprofv3 kernel trace + stats of bench.py -> per-kernel step breakdown, the GEMM
# family per shape (HIP events), and the GEMM / attention micro-benchmarks.  Each GPU step has its own time limit.
#   usage (gpurun): bash tools/gpu_profile.sh [tag]      outputs: gpurun_out/<tag>_*
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-prof}
mkdir -p gpurun_out
rm -rf gpurun_out/${T}_trace
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_trace -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-roofline --epochs 0 --no-extra ${BENCH_ARGS:-} > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err \
    || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
cat gpurun_out/${T}_bench.json
python3 tools/step_breakdown.py $(find gpurun_out/${T}_trace -name '*kernel_trace.csv' | head -1) \
    $(python3 -c "import json;print(json.load(open('gpurun_out/${T}_bench.json')).get('family_launches_per_step', ${LPS:-2314}))") 2 \
    > gpurun_out/${T}_breakdown.txt && head -40 gpurun_out/${T}_breakdown.txt
[ "${SHAPES:-1}" = 1 ] && { timeout -k 10 300 python3 tools/shape_prof.py > gpurun_out/${T}_shapes.txt 2>&1 || exit 1; head -40 gpurun_out/${T}_shapes.txt; }
[ "${GEMM:-0}" = 1 ] && { GEMM_LIB=1 timeout -k 10 300 python3 tools/gemm_bench.py > gpurun_out/${T}_gemm.txt 2>&1 || exit 1; cat gpurun_out/${T}_gemm.txt; }
[ "${ATTN:-0}" = 1 ] && { timeout -k 10 200 python3 tools/attn_bench.py > gpurun_out/${T}_attn.txt 2>&1 || exit 1; cat gpurun_out/${T}_attn.txt; }
exit 0
