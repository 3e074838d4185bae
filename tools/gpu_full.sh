#!/bin/bash
# One gpurun call for the round's evidence: GPU parity tests -> bench (with roofline + cpu_baseline) ->
# rocprofv3 kernel-trace/stats of the same bench -> two PMC passes (FETCH_SIZE, WRITE_SIZE) for HBM traffic.
# Every GPU step has its own time limit; the script stops at the first failure.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
STEPS=${BENCH_STEPS:-5}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -s --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; grep -E "passed|failed|Error" gpurun_out/pytest_gpu.log | tail -15
  [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 900 python bench.py --steps $STEPS --warmup 2 ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
echo "bench rc=$rc"; cat gpurun_out/bench.json; [ $rc -ne 0 ] && { tail -20 gpurun_out/bench.err; exit $rc; }
rm -rf gpurun_out/prof gpurun_out/pmc_fetch gpurun_out/pmc_write
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-roofline --epochs 0 --no-extra > gpurun_out/prof_bench.json 2> gpurun_out/prof_bench.err; rc=$?
echo "rocprof rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/prof_bench.err; exit $rc; }
[ "${SKIP_PMC:-0}" == 1 ] && exit 0
for C in FETCH_SIZE WRITE_SIZE; do
  D=gpurun_out/pmc_$(echo $C | cut -d_ -f1 | tr A-Z a-z)
  timeout -k 10 600 rocprofv3 --pmc $C --kernel-trace --kernel-include-regex "gemm" --output-format csv -d $D -o run -- \
      python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-roofline --epochs 0 --no-extra > $D.json 2> $D.err; rc=$?
  echo "pmc $C rc=$rc"; [ $rc -ne 0 ] && { tail -20 $D.err; exit $rc; }
done
exit 0
