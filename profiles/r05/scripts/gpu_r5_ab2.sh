#!/bin/bash
# r5: live-values parity after the kernel split, then the snapshot kernel A/B against the r4 build
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
mkdir -p gpurun_out/r5ab2
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "live or narrow or dist_plan" > gpurun_out/r5ab2/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 2 gpurun_out/r5ab2/pytest.log; [ $rc -eq 0 ] || exit $rc
CFGS="cop20k_k32 cop20kirr_k32" ROUNDS=3 LIBS="libsmfv_ab.so libsmfv.so" bash scripts/ab_lib.sh
