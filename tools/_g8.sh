mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_layers.py > gpurun_out/pytest_k.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_k.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAILED|rel" gpurun_out/pytest_k.log | head -20; exit $rc; }
GEMM_VARIANTS=0,30,32 timeout -k 10 300 python -u tools/gemm_bench.py > gpurun_out/gemm_bench.txt 2>&1; rc=$?
cat gpurun_out/gemm_bench.txt
exit $rc
