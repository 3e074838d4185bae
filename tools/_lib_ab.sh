#!/bin/bash
# Same-box A/B of two builds of libpso_amd.so on the C2 step: ab/libpso_amd_prev.so (previous commit) vs the tree's.
mkdir -p gpurun_out
for L in prev cur prev cur; do
  if [ $L = prev ]; then export PSO_LIB_PATH=$PWD/ab/libpso_amd_prev.so; else unset PSO_LIB_PATH; fi
  timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline \
      > gpurun_out/lab_$L.json 2> gpurun_out/lab_$L.err || exit $?
  echo "lib $L: $(python -c "import json;d=json.load(open('gpurun_out/lab_$L.json'));print(d['value'],d['ms_per_step'])")"
done
