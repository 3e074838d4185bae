#!/bin/bash
# Same-box A/B of GEMM dispatch knobs on the C2 step: VARS="0 400 1600" (variant + 100 * raster group rows)
mkdir -p gpurun_out
for v in ${VARS:-0 400 1600}; do
  PSO_BENCH_GEMM_VARIANT=$v timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline \
      > gpurun_out/var_$v.json 2> gpurun_out/var_$v.err || exit $?
  echo "gemm variant $v: $(python -c "import json;d=json.load(open('gpurun_out/var_$v.json'));print(d['value'],d['ms_per_step'])")"
done
