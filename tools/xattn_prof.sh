#!/bin/bash
# Kernel durations (rocprofv3 kernel trace, no Python launch overhead) of the cross-attention kernels on the SDXL
# 77-key shapes: tools/attn_bench.py (ATTN_CROSS_ONLY) under the profiler, averaged per (kernel, grid) by
# tools/trace_by_grid.py.   usage (gpurun): ATTN_IMAGES=16 ATTN_VARIANTS=990000,0 bash tools/xattn_prof.sh [tag]
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-xattn}
mkdir -p gpurun_out && rm -rf gpurun_out/${T}_trace
[ -z "${ATTN_SHAPE:-}" ] && export ATTN_CROSS_ONLY=1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_trace -o run -- \
    python3 tools/attn_bench.py > gpurun_out/${T}_bench.txt 2>&1 || { tail -20 gpurun_out/${T}_bench.txt; exit 1; }
python3 tools/trace_by_grid.py gpurun_out/${T}_trace attn > gpurun_out/${T}_kernels.txt && cat gpurun_out/${T}_kernels.txt
python3 tools/trace_by_grid.py gpurun_out/${T}_trace reduce_splits >> gpurun_out/${T}_kernels.txt
