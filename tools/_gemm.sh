mkdir -p gpurun_out
GEMM_VARIANTS=${GEMM_VARIANTS:-0,12,14,16,17,18,19} timeout -k 10 300 python tools/gemm_bench.py > gpurun_out/gemm_bench.txt 2>&1; rc=$?
cat gpurun_out/gemm_bench.txt
exit $rc
