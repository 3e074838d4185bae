#!/bin/bash
# PMC passes over the flash-attention micro-benchmark (one rocprofv3 run per counter group, each under its own limit).
#   usage (GPU box): tools/attn_pmc.sh [outdir]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/attn_pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp ATTN_IMAGES=${ATTN_IMAGES:-16} ATTN_VARIANTS=${ATTN_VARIANTS:-0}
passes=(
  "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS"
  "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_MISC"
  "SQ_INSTS_VALU_TRANS_F32 SQ_WAIT_INST_LDS SQ_INST_LEVEL_LDS SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_VMEM SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE"
)
i=0
for p in "${passes[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $p --output-format csv -d "$OUT/p$i" -o pmc -- python3 tools/attn_bench.py > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
