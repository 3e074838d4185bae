mkdir -p gpurun_out
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench11.json 2> gpurun_out/bench11.err; rc=$?
cat gpurun_out/bench11.json
if [ $rc -ne 0 ]; then tail -20 gpurun_out/bench11.err; exit $rc; fi
BENCH_STEPS=2 bash tools/prof_bench.sh
