#!/bin/bash
# One gpurun call: GPU tests, then (only if the tests did not fault / time out) a short bench.
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -s > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
grep -E "passed|failed|rel err|rel=|Error" gpurun_out/pytest_gpu.log | tail -30
if [ $rc -ge 124 ]; then echo "stopping after pytest rc=$rc"; exit $rc; fi
timeout -k 10 900 python bench.py --steps ${BENCH_STEPS:-3} --warmup 1 ${BENCH_ARGS:---no-cpu-baseline} > gpurun_out/bench.json 2> gpurun_out/bench.err
brc=$?
echo "bench rc=$brc"; tail -5 gpurun_out/bench.err; cat gpurun_out/bench.json
exit $brc
