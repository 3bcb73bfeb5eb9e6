#!/bin/bash
# r6 A/B: row-pair admission on the irregular stand-in (SMFV_PAIR_SLACK:
# batches a pair may run past the tile's longest row, default 1;
# SMFV_PAIR_LEN: longest second row, default 56), same binary, alternated.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"
OUT=$ROOT/gpurun_out/r6_pairs; mkdir -p "$OUT"
A="--no-cpu-baseline --no-vendor --no-rebind --no-copy-floor --no-warm"
for r in 1 2; do
  for v in "1 56" "0 56" "2 56" "1 40" "1 62" "2 62"; do
    set -- $v
    SMFV_PAIR_SLACK=$1 SMFV_PAIR_LEN=$2 timeout -k 10 300 python bench.py --config cop20kirr_k32 $A > "$OUT/irr_s$1_l$2_$r.json" 2> "$OUT/irr_s$1_l$2_$r.log"
    rc=$?; [ $rc -eq 0 ] || { echo "bench s$1 l$2 rc=$rc"; exit $rc; }
    python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['ms_per_step'], d['check']['ok'], d['plan']['tiles'], d['plan']['paired_rows'])" "$OUT/irr_s$1_l$2_$r.json" "slack=$1 len=$2 $r"
  done
done
