mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-roofline > gpurun_out/prof_bench.json 2> gpurun_out/prof_bench.err; rc=$?
echo "rocprof rc=$rc"; cat gpurun_out/prof_bench.json; [ $rc -ne 0 ] && { tail -20 gpurun_out/prof_bench.err; exit $rc; }
python tools/step_breakdown.py $(find gpurun_out/prof -name '*kernel_trace.csv' | head -1) ${LPS:-2450} 2 > gpurun_out/breakdown.txt
cat gpurun_out/breakdown.txt
