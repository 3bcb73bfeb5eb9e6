#!/bin/bash
# Lab: PMC passes over lab_spmm (one counter group per pass, kernel trace only).
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; OUT=$ROOT/gpurun_out/labpmc_${TAG:-x}; mkdir -p $OUT
python -c "
import sys; sys.path.insert(0,'.')
from sparsematrixmultiplicationmpi_amd import inputs
inputs.write_csr_bin('/tmp/cop.bin', inputs.cop20k_surrogate())" || exit 1
export TMPDIR=/tmp
SETS=${PMC_SETS:-"SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS;SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL;SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_VMEM_TA_ADDR_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_THREAD_CYCLES_VALU SQ_WAVES"}
IFS=';' read -r -a G <<< "$SETS"
i=0
for ctrs in "${G[@]}"; do
  i=$((i+1))
  (cd /tmp && timeout -k 5 90 rocprofv3 --kernel-trace --pmc $ctrs -d $OUT/p$i -o pmc --output-format csv \
     -- $ROOT/scripts/micro/${LAB_BIN:-lab_spmm} /tmp/cop.bin ${LAB_REPS:-20} > $OUT/p$i.log 2>&1)
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/p$i.log; exit $rc; }
done
python scripts/pmc_summary.py $OUT ${PMC_FILTER:-} > $OUT/summary.txt; cat $OUT/summary.txt
