#!/bin/bash
# A/B of the tiled kernels on one box: k_rows_cs (column-streamed tiles) vs
# k_rows_ws, alternating, each run checked bit-exact by bench.py.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out/ab_cs
mkdir -p "$OUT"
CFGS=${CFGS:-cop20k_k32}
REPS=${REPS:-2}
for cfg in $CFGS; do
  for r in $(seq 1 $REPS); do
    for k in ${KERNELS:-cs ws}; do
      timeout -k 10 240 python bench.py --config $cfg --tiled-kernel $k --no-cpu-baseline --no-vendor \
          --no-copy-floor ${BENCH_ARGS:-} > "$OUT/${cfg}_${k}_$r.log" 2>&1
      rc=$?; [ $rc -eq 0 ] || { echo "$cfg $k rc=$rc"; tail -n 5 "$OUT/${cfg}_${k}_$r.log"; exit $rc; }
      tail -n 1 "$OUT/${cfg}_${k}_$r.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg', '$k', d['ms_per_step']*1000, 'us', d['roofline']['frac'], d['roofline']['kernel'], d['check']['ok'], d['check']['max_abs_diff'], d['plan'].get('tiles'))"
    done
  done
done
