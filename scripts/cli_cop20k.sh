#!/bin/bash
# End-to-end CLI run (smfv_main, the SC/main.cpp drop-in) on a cop20k_A
# surrogate written as a Matrix Market file: the reference's own timing
# lines, each variant's FIRST call (no warm-up), with SMFV_TIMING=1 stage
# lines when set.  Beside it, the reference's own kernels (oracle/_ref, SC
# sources compiled unmodified) in the same order on 16 host ranks: first
# call (--reps 1, what SC/main.cpp prints) and median of 5.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; OUT=$ROOT/gpurun_out; mkdir -p $OUT
MAT=${MAT:-cop20k}   # cop20k | cop20k_irr
python -c "
import sparsematrixmultiplicationmpi_amd as smfv
from sparsematrixmultiplicationmpi_amd import inputs
A = smfv.cop20k_surrogate() if '$MAT' == 'cop20k' else inputs.cop20k_irregular_surrogate()
smfv.writeMatrixMarketFile('/tmp/$MAT.mtx', A, symmetric=True)
inputs.write_csr_bin('/tmp/$MAT.bin', A)" || exit 1
# one GPU per rank: np > 1 needs as many GPUs (RCCL refuses or hangs on a shared device)
for np in ${NPS:-1}; do
  timeout -k 10 120 /opt/conda/bin/mpiexec -launcher fork -n $np ./sparsematrixmultiplicationmpi_amd/smfv_main ${K:-32} /tmp/$MAT.mtx > $OUT/cli_${MAT}_np$np.log 2>&1
  rc=$?; echo "np $np rc=$rc"; cat $OUT/cli_${MAT}_np$np.log; [ $rc -eq 0 ] || exit $rc
done
if [ -x oracle/_ref/ref_driver ]; then
  for reps in 1 5; do
    timeout -k 10 300 /opt/conda/bin/mpiexec -launcher fork -n 16 oracle/_ref/ref_driver /tmp/$MAT.bin ${K:-32} --reps $reps > $OUT/ref_${MAT}_np16_reps$reps.log 2>&1
    rc=$?; echo "reference np 16 reps $reps rc=$rc"; grep -E "time|Results" $OUT/ref_${MAT}_np16_reps$reps.log
  done
fi
