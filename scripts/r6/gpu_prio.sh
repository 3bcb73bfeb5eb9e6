#!/bin/bash
# r6 A/B: k_rows_ws wave priorities (SMFV_WS_PRIO="LC": loaders L, compute C;
# the kernel's default 30), same binary, alternated on one box.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"
OUT=$ROOT/gpurun_out/r6_prio; mkdir -p "$OUT"
A="--no-cpu-baseline --no-vendor --no-rebind --no-copy-floor --no-warm"
for r in 1 2; do
  for cfg in cop20k_k32 cop20kirr_k32; do
    for v in 30 20 31 32 21 10; do
      SMFV_WS_PRIO=$v timeout -k 10 300 python bench.py --config $cfg $A > "$OUT/${cfg}_${v}_$r.json" 2> "$OUT/${cfg}_${v}_$r.log"
      rc=$?; [ $rc -eq 0 ] || { echo "bench $cfg $v rc=$rc"; exit $rc; }
      python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['ms_per_step'], d['check']['ok'])" "$OUT/${cfg}_${v}_$r.json" "$cfg prio=$v $r"
    done
  done
done
