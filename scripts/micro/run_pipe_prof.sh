#!/bin/bash
# Lab: phase profile of k_rows_pipe on the cop20k surrogate (K=32).
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; OUT=$ROOT/gpurun_out; mkdir -p $OUT
python -c "
import sys; sys.path.insert(0,'.')
from sparsematrixmultiplicationmpi_amd import inputs
inputs.write_csr_bin('/tmp/cop.bin', inputs.cop20k_surrogate())" || exit 1
timeout -k 10 120 scripts/micro/lab_pipe_prof /tmp/cop.bin 32 $OUT/pipe_prof.bin > $OUT/pipe_prof.log 2>&1; rc=$?
cat $OUT/pipe_prof.log; [ $rc -eq 0 ] || exit $rc
python scripts/micro/prof_summary.py $OUT/pipe_prof.bin
