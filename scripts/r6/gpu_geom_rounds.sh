#!/bin/bash
# r6 A/B: small tiled plans take geometry 2 where it runs fewer rounds of
# units (default) against the previous rule (SMFV_WS_GEOM_ROUNDS=0), same
# binary, alternated: ROWWISE rank-plan projections at p = 8 / 4 / 2 on both
# cop20k stand-ins, parity of every rank plan at full size first.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"
OUT=$ROOT/gpurun_out/r6_geom; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_rank_plans_fullsize.py -k "ROWWISE" > "$OUT/pytest_ranks.log" 2>&1
rc=$?; echo "pytest ranks rc=$rc"; tail -n 2 "$OUT/pytest_ranks.log"; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for cfg in cop20k_k32 cop20kirr_k32; do
    for p in 8 4; do
      for v in 1 0; do
        SMFV_WS_GEOM_ROUNDS=$v timeout -k 10 300 python bench.py --config $cfg --rank-plans $p --steps 100 --warmup 10 \
            > "$OUT/rw_${cfg}_p${p}_g${v}_$r.json" 2> "$OUT/rw_${cfg}_p${p}_g${v}_$r.log"
        rc=$?; [ $rc -eq 0 ] || { echo "bench $cfg p$p g$v rc=$rc"; exit $rc; }
        python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['rank_local_us_max'], d['rank_local_us_min'], d['check']['ok'], [(x['tiles'], x['ws_geom']) for x in d['ranks']])" "$OUT/rw_${cfg}_p${p}_g${v}_$r.json" "$cfg p$p rounds=$v $r"
      done
    done
  done
done
