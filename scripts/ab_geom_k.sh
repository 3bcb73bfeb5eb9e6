#!/bin/bash
# geometry 1 vs 3 (bench.py --tiled-kernel ws1 / ws3) at K = 64 / 128 (and
# the headline K = 32 as a control), alternating on one box
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/ab_geom_k
for cfg in ${CFGS:-cop20k_k128 cop20k_k32}; do
 for r in 1 2 3; do
  for g in ws1 ws3; do
    timeout -k 10 200 python bench.py --config $cfg --tiled-kernel $g --no-cpu-baseline --no-vendor --no-copy-floor --no-rebind ${EXTRA:-} \
      > gpurun_out/ab_geom_k/${cfg}_${g}_$r.json 2> gpurun_out/ab_geom_k/${cfg}_${g}_$r.log || exit $?
    tail -n 1 gpurun_out/ab_geom_k/${cfg}_${g}_$r.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg $g', round(d['ms_per_step']*1e3, 3), d['roofline']['frac'], d['check']['ok'], d['check']['max_abs_diff'])"
  done
 done
done
