mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q -x > gpurun_out/t13.log 2>&1; rc=$?
tail -3 gpurun_out/t13.log
[ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/t13.log | head -20; exit $rc; }
timeout -k 10 300 python tools/tn_bench.py 2>&1 | grep -v amdgpu.ids; rc=$?
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/shape_prof.py > gpurun_out/shape_prof.txt 2>&1; rc=$?
head -30 gpurun_out/shape_prof.txt
exit $rc
