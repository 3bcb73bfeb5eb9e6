#!/bin/bash
# Lab: PMC counter groups for tiled-kernel ablation modes (SMFV_TILED_ABLATE).
# Usage: MODES="0 6" bash scripts/gpu_pmc_modes.sh ; stops at the first crash/timeout.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
export TMPDIR=/tmp
cd /tmp
SETS=${PMC_SETS:-"SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES;SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS;SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_LDS_ADDR_CONFLICT;SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY"}
IFS=';' read -r -a GROUPS_ARR <<< "$SETS"
for mode in ${MODES:-0 6}; do
  mkdir -p "$OUT/pmcm_$mode"
  i=0
  for ctrs in "${GROUPS_ARR[@]}"; do
    i=$((i+1))
    SMFV_TILED_ABLATE=$mode timeout -k 10 300 rocprofv3 --kernel-trace --pmc $ctrs -d "$OUT/pmcm_$mode/p$i" -o pmc --output-format csv \
       -- python3 "$ROOT/bench.py" --no-cpu-baseline --steps 10 --warmup 2 --tiles force > "$OUT/pmcm_$mode/p$i.log" 2>&1
    rc=$?; echo "mode $mode pass $i ($ctrs) rc=$rc"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  done
  python3 "$ROOT/scripts/pmc_summary.py" "$OUT/pmcm_$mode" k_rows_pipe
done
