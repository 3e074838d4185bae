#!/bin/bash
# short-KV (cross-attention) backward A/B under rocprofv3: variant 70 = the dQ + dK/dV launches, 0 = attn_bwd_x_kernel
# with the automatic query splits, 10000*qs = forced splits.  usage (gpurun): XB_VARIANTS="70,0,20000" bash tools/xb_run.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for n in ${XB_IMAGES:-16 8 2}; do
  ATTN_IMAGES=$n ATTN_VARIANTS=${XB_VARIANTS:-70,0} bash tools/xattn_prof.sh xb$n > /dev/null || exit 1
  echo "== $n images"
  python3 tools/trace_by_grid.py gpurun_out/xb${n}_trace attn_bwd
  python3 tools/trace_by_grid.py gpurun_out/xb${n}_trace reduce_splits
done
