mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_kernels.py -q -x > gpurun_out/t16.log 2>&1; rc=$?
tail -2 gpurun_out/t16.log
[ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/t16.log | head -20; exit $rc; }
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
cat gpurun_out/bench.json; [ $rc -ne 0 ] && { tail -20 gpurun_out/bench.err; exit $rc; }
timeout -k 10 300 python tools/shape_prof.py > gpurun_out/shape_prof.txt 2>&1; rc=$?
head -45 gpurun_out/shape_prof.txt
exit $rc
