#!/bin/bash
# Lab: k_rows_pipe ablations (SMFV_TILED_ABLATE) on the bench workload.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; OUT=$ROOT/gpurun_out; mkdir -p $OUT
for mode in ${MODES:-0 4 5 6 7 8 9}; do
  SMFV_TILED_ABLATE=$mode timeout -k 10 120 python bench.py --no-cpu-baseline --steps 100 --warmup 10 ${BENCH_ARGS:-} > $OUT/abl_$mode.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "mode $mode rc=$rc"; tail -5 $OUT/abl_$mode.log; exit $rc; }
  python -c "
import json,sys; d=json.loads(open('$OUT/abl_$mode.log').read().strip().splitlines()[-1])
print('mode $mode', 'cold us %.2f'%(d['roofline']['avg_launch_ms']*1e3), 'warm us %.2f'%(d['warm']['avg_launch_ms']*1e3))"
done
