#!/bin/bash
# End-to-end CLI run (smfv_main, the SC/main.cpp drop-in) on the cop20k_A
# surrogate written as a Matrix Market file: the reference's own timing lines.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; OUT=$ROOT/gpurun_out; mkdir -p $OUT
python -c "
import sparsematrixmultiplicationmpi_amd as smfv
smfv.writeMatrixMarketFile('/tmp/cop20k_surrogate.mtx', smfv.cop20k_surrogate(), symmetric=True)" || exit 1
# one GPU per rank: np > 1 needs as many GPUs (RCCL refuses or hangs on a shared device)
for np in ${NPS:-1}; do
  timeout -k 10 120 /opt/conda/bin/mpiexec -launcher fork -n $np ./sparsematrixmultiplicationmpi_amd/smfv_main ${K:-32} /tmp/cop20k_surrogate.mtx > $OUT/cli_np$np.log 2>&1
  rc=$?; echo "np $np rc=$rc"; cat $OUT/cli_np$np.log; [ $rc -eq 0 ] || exit $rc
done
