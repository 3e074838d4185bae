#!/bin/bash
# Same-box A/B of the attention row-sum forms: micro-bench in both orders, then the C2 step with each.
mkdir -p gpurun_out
ATTN_VARIANTS=100,0,100,0 timeout -k 10 200 python tools/attn_bench.py > gpurun_out/attn_ab.log 2>&1 || exit $?
cat gpurun_out/attn_ab.log
for v in 0 100 0 100; do
  PSO_BENCH_ATTN_VARIANT=$v timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline \
      > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || exit $?
  echo "attn variant $v: $(python -c "import json;d=json.load(open('gpurun_out/ab_$v.json'));print(d['value'],d['ms_per_step'])")"
done
