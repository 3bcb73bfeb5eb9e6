#!/bin/bash
# r5: narrow-team tiles (k_rows_wsn) for a ColumnWise rank's K/p window --
# parity, then the rank-plan projections at p = 8 / 4 (K/p = 4 / 8) against
# k_rows_ws's NARROW form (--tiled-kernel ws1), alternating on one box.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out/r5wsn; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "narrow or column" > "$OUT/pytest_parity.log" 2>&1
rc=$?; echo "pytest parity rc=$rc"; tail -n 2 "$OUT/pytest_parity.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_rank_plans_fullsize.py tests/test_gpu_dist_parity.py tests/test_gpu_large_goldens.py -k "COLUMNWISE or rank_plans or building" \
    > "$OUT/pytest_ranks.log" 2>&1
rc=$?; echo "pytest ranks rc=$rc"; tail -n 2 "$OUT/pytest_ranks.log"; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for cfg in cop20k_k32 cop20kirr_k32; do
    for p in 8 4; do
      for tk in auto ws1; do
        timeout -k 10 300 python bench.py --config $cfg --variant COLUMNWISE --rank-plans $p --tiled-kernel $tk \
            --steps 100 --warmup 10 > "$OUT/cw_${cfg}_p${p}_${tk}_$r.json" 2> "$OUT/cw_${cfg}_p${p}_${tk}_$r.log" || exit $?
        python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['rank_local_us_max'], d['rank_local_us_min'], d['check']['ok'], d['ranks'][0]['tiles'])" "$OUT/cw_${cfg}_p${p}_${tk}_$r.json" "$cfg p$p $tk"
      done
    done
  done
done
