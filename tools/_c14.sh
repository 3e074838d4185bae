mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_trainer.py -q -x -s > gpurun_out/t14.log 2>&1; rc=$?
grep -E "batched|passed|failed" gpurun_out/t14.log
[ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/t14.log | head -20; exit $rc; }
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
cat gpurun_out/bench.json; [ $rc -ne 0 ] && { tail -20 gpurun_out/bench.err; exit $rc; }
rm -rf gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-roofline > gpurun_out/prof_bench.json 2> gpurun_out/prof_bench.err; rc=$?
echo "rocprof rc=$rc"; head -25 gpurun_out/prof/run_kernel_stats.csv | cut -c1-150
exit $rc
