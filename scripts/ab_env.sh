#!/bin/bash
# A/B of one env knob on the headline bench: VAR=SMFV_WS_RSX VALUES="0 4" bash scripts/ab_env.sh
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; OUT=$ROOT/gpurun_out; mkdir -p $OUT
for v in $VALUES; do
  env $VAR=$v timeout -k 10 120 python bench.py --no-cpu-baseline --steps 200 --warmup 20 ${BENCH_ARGS:-} > $OUT/ab_${VAR}_$v.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$VAR=$v rc=$rc"; tail -5 $OUT/ab_${VAR}_$v.log; exit $rc; }
  python -c "
import json; d=json.loads(open('$OUT/ab_${VAR}_$v.log').read().strip().splitlines()[-1])
print('$VAR=$v', 'cold us %.2f'%(d['roofline']['avg_launch_ms']*1e3), 'warm us %.2f'%(d['warm']['avg_launch_ms']*1e3), d['value'])"
done
