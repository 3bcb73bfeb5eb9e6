#!/bin/bash
# r5: k_rows_wsn with batches of 4 entries (this tree) against batches of 8
# (libsmfv_ab.so, the previous build): parity, then the ColumnWise rank-plan
# projections at p = 8 / 4 (K/p = 4 / 8), alternating on one box.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out/r5wsn4; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "narrow or column or row_pair" > "$OUT/pytest_parity.log" 2>&1
rc=$?; echo "pytest parity rc=$rc"; tail -n 2 "$OUT/pytest_parity.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_rank_plans_fullsize.py -k "COLUMNWISE" > "$OUT/pytest_ranks.log" 2>&1
rc=$?; echo "pytest ranks rc=$rc"; tail -n 2 "$OUT/pytest_ranks.log"; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for cfg in cop20k_k32 cop20kirr_k32; do
    for p in 8 4; do
      for lib in libsmfv.so libsmfv_ab.so; do
        SMFV_LIB=$lib timeout -k 10 300 python bench.py --config $cfg --variant COLUMNWISE --rank-plans $p \
            --steps 100 --warmup 10 > "$OUT/cw_${cfg}_p${p}_${lib%.so}_$r.json" 2> "$OUT/cw_${cfg}_p${p}_${lib%.so}_$r.log" || exit $?
        python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['rank_local_us_max'], d['rank_local_us_min'], d['check']['ok'], d['ranks'][0]['tiles'])" "$OUT/cw_${cfg}_p${p}_${lib%.so}_$r.json" "$cfg p$p $lib"
      done
    done
  done
done
