#!/bin/bash
# r6: full-size rank plans at every p including 3 and 5 (uneven ColumnWise
# windows), one GPU process under its own limit.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"
OUT=$ROOT/gpurun_out/r6rankodd; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_rank_plans_fullsize.py > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 5 "$OUT/pytest.log"; exit $rc
