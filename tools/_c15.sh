mkdir -p gpurun_out
GEMM_VARIANTS=0,4,5,1,2,3,6,7,8,9 timeout -k 10 600 python tools/gemm_bench.py > gpurun_out/gemm_bench.txt 2>&1; rc=$?
cat gpurun_out/gemm_bench.txt | grep -v amdgpu
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/shape_prof.py > gpurun_out/shape_prof.txt 2>&1; rc=$?
head -45 gpurun_out/shape_prof.txt
exit $rc
