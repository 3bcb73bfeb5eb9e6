#!/bin/bash
# Lab: candidate kernels on the cop20k surrogate (scripts/micro/lab_spmm.hip).
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; OUT=$ROOT/gpurun_out; mkdir -p $OUT
[ -f /tmp/cop.bin ] || python -c "
import sys; sys.path.insert(0,'.')
from sparsematrixmultiplicationmpi_amd import inputs
inputs.write_csr_bin('/tmp/cop.bin', inputs.cop20k_surrogate())" || exit 1
timeout -k 10 ${LAB_TIMEOUT:-120} scripts/micro/${LAB_BIN:-lab_spmm} /tmp/cop.bin ${LAB_REPS:-200} 2>&1 | tee $OUT/lab_${TAG:-x}.log
