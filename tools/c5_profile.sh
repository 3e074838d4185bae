cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for m in bf16 fp8; do
  F=""; [ $m = fp8 ] && F="--fp8"
  rm -rf gpurun_out/c5_$m
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5_$m -o run -- python3 tools/db_bench.py --steps 4 --warmup 2 $F > gpurun_out/c5_$m.json 2> gpurun_out/c5_$m.err || exit 1
done
