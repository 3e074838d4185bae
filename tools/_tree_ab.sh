#!/bin/bash
# Same-box A/B of the C2 step: ab/prev (a snapshot of the previous commit: sources + its built library) vs this tree.
mkdir -p gpurun_out
R=$PWD
for L in prev cur prev cur; do
  if [ $L = prev ]; then D=$R/ab/prev; else D=$R; fi
  (cd $D && timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline) \
      > gpurun_out/tab_$L.json 2> gpurun_out/tab_$L.err || exit $?
  echo "tree $L: $(python -c "import json;d=json.load(open('gpurun_out/tab_$L.json'));print(d['value'],d['ms_per_step'])")"
done
