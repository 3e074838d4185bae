mkdir -p gpurun_out
timeout -k 10 300 python tools/shape_prof.py > gpurun_out/shape_prof.txt 2>&1; rc=$?
tail -62 gpurun_out/shape_prof.txt
[ $rc -ne 0 ] && exit $rc
GEMM_VARIANTS=0,4,5,1,2,3 timeout -k 10 300 python tools/gemm_bench.py > gpurun_out/gemm_bench.txt 2>&1; rc=$?
cat gpurun_out/gemm_bench.txt
exit $rc
