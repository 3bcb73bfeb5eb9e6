#!/bin/bash
# bind kernel A/B: NEW (libsmfv.so) vs OLD (libsmfv_lab.so), alternating on one box
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/ab_bind_lab
for cfg in ${CFGS:-cop20k_k32 cop20kirr_k32}; do
 for r in 1 2 3; do
  for lab in 0 1; do
    SMFV_LAB=$lab timeout -k 10 200 python bench.py --config $cfg --no-cpu-baseline --no-vendor --no-copy-floor \
      > gpurun_out/ab_bind_lab/${cfg}_${lab}_$r.json 2> gpurun_out/ab_bind_lab/${cfg}_${lab}_$r.log || exit $?
    tail -n 1 gpurun_out/ab_bind_lab/${cfg}_${lab}_$r.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); rb=d['plan']['rebind_each_step']; print('$cfg', 'old' if $lab else 'new', round(d['ms_per_step']*1e3,2), 'bind', round(rb['bind_ms']*1e3,2), 'b+e', round(rb['bind_plus_execute_ms']*1e3,2), d['check']['ok'])"
  done
 done
done
