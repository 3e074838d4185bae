mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
cat gpurun_out/bench.json; [ $rc -ne 0 ] && { tail -20 gpurun_out/bench.err; exit $rc; }
timeout -k 10 300 python tools/shape_prof.py > gpurun_out/shape_prof.txt 2>&1; rc=$?
head -40 gpurun_out/shape_prof.txt
[ $rc -ne 0 ] && exit $rc
if [ -n "$GEMM" ]; then
  timeout -k 10 300 python tools/gemm_bench.py > gpurun_out/gemm_bench.txt 2>&1; rc=$?
  cat gpurun_out/gemm_bench.txt
fi
exit $rc
