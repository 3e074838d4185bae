# A/B of the C2 bench under two GEMM variants in one call: BENCH_AB="0 41"
mkdir -p gpurun_out
for v in ${BENCH_AB:-0 41}; do
  echo "variant $v"; PSO_BENCH_GEMM_VARIANT=$v timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline 2>/dev/null | cut -c1-150 || exit 1
done
