#!/bin/bash
# r6: the live-values X >= 4 GiB fallback test, then LDS bank-conflict
# counters of k_rows_wsn (ColumnWise rank 0 of p = 8, K/p = 4) with
# bank-coloured slots and with first-use slots (SMFV_WSN_FIRST_USE_SLOTS=1),
# one counter group per run, kernel trace only.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"
OUT=$ROOT/gpurun_out/r6_wsnpmc; mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "x_over_4gib or mix_floor" > "$OUT/pytest_live4g.log" 2>&1
rc=$?; echo "pytest live>4GiB rc=$rc"; tail -n 2 "$OUT/pytest_live4g.log"; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
cd /tmp
for v in colour first; do
  if [ $v = first ]; then export SMFV_WSN_FIRST_USE_SLOTS=1; else unset SMFV_WSN_FIRST_USE_SLOTS; fi
  timeout -s KILL 180 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAVE_CYCLES \
      -d "$OUT/pmc_$v" -o pmc --output-format csv -- python3 "$ROOT/bench.py" --config cop20k_k32 --variant COLUMNWISE \
      --rank-plans 8 --rank-only 0 --steps 20 --warmup 2 --cold-bytes 1e8 > "$OUT/pmc_$v.log" 2>&1
  rc=$?; echo "pmc $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
unset SMFV_WSN_FIRST_USE_SLOTS
