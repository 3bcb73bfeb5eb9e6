#!/bin/bash
# r6 A/B: k_rows_wsn plans with bank-coloured image slots (default) against
# first-use slots (SMFV_WSN_FIRST_USE_SLOTS=1), same binary, alternated:
# parity first, then ColumnWise rank-plan projections at p = 8 / 4.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"
OUT=$ROOT/gpurun_out/r6_wsn; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "narrow" > "$OUT/pytest_parity.log" 2>&1
rc=$?; echo "pytest parity rc=$rc"; tail -n 2 "$OUT/pytest_parity.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_rank_plans_fullsize.py -k "COLUMNWISE" > "$OUT/pytest_ranks.log" 2>&1
rc=$?; echo "pytest ranks rc=$rc"; tail -n 2 "$OUT/pytest_ranks.log"; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for cfg in cop20k_k32 cop20kirr_k32; do
    for p in 8 4; do
      for v in colour first; do
        if [ $v = first ]; then export SMFV_WSN_FIRST_USE_SLOTS=1; else unset SMFV_WSN_FIRST_USE_SLOTS; fi
        timeout -k 10 300 python bench.py --config $cfg --variant COLUMNWISE --rank-plans $p --steps 100 --warmup 10 \
            > "$OUT/cw_${cfg}_p${p}_${v}_$r.json" 2> "$OUT/cw_${cfg}_p${p}_${v}_$r.log"
        rc=$?; [ $rc -eq 0 ] || { echo "bench $cfg p$p $v rc=$rc"; exit $rc; }
        python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['rank_local_us_max'], d['rank_local_us_min'], d['check']['ok'], d['ranks'][0]['tiles'])" "$OUT/cw_${cfg}_p${p}_${v}_$r.json" "$cfg p$p $v $r"
      done
    done
  done
done
unset SMFV_WSN_FIRST_USE_SLOTS
