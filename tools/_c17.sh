mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_kernels.py -q -x -k "variant or skinny or tn or splitk or vs_fp32" > gpurun_out/t17.log 2>&1; rc=$?
tail -2 gpurun_out/t17.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/t17.log | head -20; exit $rc; }
GEMM_VARIANTS=0,4,8,11,1,6 timeout -k 10 600 python tools/gemm_bench.py > gpurun_out/gemm_bench.txt 2>&1; rc=$?
cat gpurun_out/gemm_bench.txt | grep -v amdgpu
exit $rc
