mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_unet.py -q -x -k "tn or lora or grad or unet or skinny" --timeout 200 --timeout-method thread > gpurun_out/pytest_tn.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_tn.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/pytest_tn.log | head -20; exit $rc; }
timeout -k 10 200 python tools/tn_bench.py > gpurun_out/tn_bench.txt 2>&1; rc=$?
cat gpurun_out/tn_bench.txt
exit $rc
