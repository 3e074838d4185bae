#!/bin/bash
# query-split sweep of attn_bwd_x_kernel per cross-attention level and image count (rocprofv3 kernel times)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for n in ${XB_IMAGES:-8 2}; do for L in L2 L1; do
  ATTN_SHAPE="$L cross" ATTN_IMAGES=$n ATTN_VARIANTS=${XB_VARIANTS:-0,10000,20000,30000,40000,60000,80000,120000,160000} \
      bash tools/xattn_prof.sh xq > /dev/null || exit 1
  echo "== $L cross, $n images (grid / 256 = qs * H * B)"
  python3 tools/trace_by_grid.py gpurun_out/xq_trace attn_bwd_x; python3 tools/trace_by_grid.py gpurun_out/xq_trace reduce_splits
done; done
