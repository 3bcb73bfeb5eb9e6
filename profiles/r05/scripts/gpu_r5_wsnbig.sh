#!/bin/bash
# (r5) k_rows_wsn at K/p = 4 with bigger units (703 union rows, 5,632 entries:
# 161,792 of 163,840 B of LDS): 8 XCD parts (521 stencil tiles, 3 rounds) and
# one part (WSN_ONEPART=1: 507 tiles, 2 rounds) against the current build
# (libsmfv_ab.so: 705 tiles, 3 rounds).  Parity first, then the ColumnWise
# rank-plan projections at p = 8, alternating on one box.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out/r5wsnbig; mkdir -p "$OUT"
WSN_ONEPART=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "narrow or column" > "$OUT/pytest_parity.log" 2>&1
rc=$?; echo "pytest parity rc=$rc"; tail -n 2 "$OUT/pytest_parity.log"; [ $rc -eq 0 ] || exit $rc
WSN_ONEPART=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_rank_plans_fullsize.py -k "COLUMNWISE" > "$OUT/pytest_ranks.log" 2>&1
rc=$?; echo "pytest ranks rc=$rc"; tail -n 2 "$OUT/pytest_ranks.log"; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for cfg in cop20k_k32 cop20kirr_k32; do
    for leg in one eight old; do
      case $leg in
        one) L=libsmfv.so; E=1 ;;
        eight) L=libsmfv.so; E= ;;
        old) L=libsmfv_ab.so; E= ;;
      esac
      WSN_ONEPART=$E SMFV_LIB=$L timeout -k 10 300 python bench.py --config $cfg --variant COLUMNWISE --rank-plans 8 \
          --steps 100 --warmup 10 > "$OUT/cw_${cfg}_${leg}_$r.json" 2> "$OUT/cw_${cfg}_${leg}_$r.log" || exit $?
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['rank_local_us_max'], d['rank_local_us_min'], d['check']['ok'], d['ranks'][0]['tiles'])" "$OUT/cw_${cfg}_${leg}_$r.json" "$cfg $leg"
    done
  done
done
