#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run (summary copied into profiles/ by the caller)
mkdir -p gpurun_out/prof
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
    python3 bench.py --steps ${BENCH_STEPS:-2} --warmup 1 --no-cpu-baseline --no-roofline > gpurun_out/prof_bench.json 2> gpurun_out/prof_bench.err
rc=$?
echo "rocprof rc=$rc"
find gpurun_out/prof -name "*stats*" | head
exit $rc
