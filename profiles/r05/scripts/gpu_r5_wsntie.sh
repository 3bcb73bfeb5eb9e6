#!/bin/bash
# (r5) k_rows_wsn plans at the same rounds of units: the most tiles (default)
# against the fewest (SMFV_WSN_FEW=1), ColumnWise rank-plan projections,
# alternating on one box.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out/r5wsntie; mkdir -p "$OUT"
for r in 1 2; do
  for case in "cop20k_k32 8" "cop20k_k32 4" "cop20kirr_k32 4"; do
    set -- $case
    for few in 0 1; do
      SMFV_WSN_FEW=$few timeout -k 10 300 python bench.py --config $1 --variant COLUMNWISE --rank-plans $2 \
          --steps 100 --warmup 10 > "$OUT/cw_$1_p$2_few${few}_$r.json" 2> "$OUT/cw_$1_p$2_few${few}_$r.log" || exit $?
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['rank_local_us_max'], d['rank_local_us_min'], d['check']['ok'], d['ranks'][0]['tiles'])" "$OUT/cw_$1_p$2_few${few}_$r.json" "$1 p$2 few=$few"
    done
  done
done
