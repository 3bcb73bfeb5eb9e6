#!/bin/bash
# (r5) k_rows_wsn tiles ordered per XCD with the smallest in the first and last
# rounds (the pipeline fill and drain, SMFV_WSN_ENDS=1) against the analysis order,
# ColumnWise rank-plan projections, alternating on one box.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out/r5wsnends; mkdir -p "$OUT"
for r in 1 2; do
  for case in "cop20k_k32 8" "cop20kirr_k32 8" "cop20k_k32 4" "cop20kirr_k32 4"; do
    set -- $case
    for few in 0 1; do
      SMFV_WSN_ENDS=$few timeout -k 10 300 python bench.py --config $1 --variant COLUMNWISE --rank-plans $2 \
          --steps 100 --warmup 10 > "$OUT/cw_$1_p$2_ends${few}_$r.json" 2> "$OUT/cw_$1_p$2_ends${few}_$r.log" || exit $?
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['rank_local_us_max'], d['rank_local_us_min'], d['check']['ok'], d['ranks'][0]['tiles'])" "$OUT/cw_$1_p$2_ends${few}_$r.json" "$1 p$2 ends=$few"
    done
  done
done
