mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/aprof
ATTN_VARIANTS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/aprof -o run -- python3 tools/attn_bench.py > gpurun_out/attn_prof.txt 2>&1; rc=$?
cat gpurun_out/attn_prof.txt
head -20 $(find gpurun_out/aprof -name '*kernel_stats.csv' | head -1) | cut -d, -f1-8
exit $rc
