#!/bin/bash
# A/B: NEW (libsmfv.so) vs OLD (libsmfv_lab.so = a copy of the previous product build), alternating
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
for cfg in cop20k_k32 cop20k_k128 cop20kirr_k32; do
 for r in 1 2; do
  for lab in 0 1; do
    SMFV_LAB=$lab timeout -k 10 200 python bench.py --config $cfg --no-cpu-baseline --no-vendor --no-copy-floor > gpurun_out/ab_${cfg}_${lab}_$r.log 2>&1 || exit $?
    tail -n 1 gpurun_out/ab_${cfg}_${lab}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg', 'old' if $lab else 'new', d['ms_per_step']*1e3, d['roofline']['frac'], d['check']['ok'], d['check']['max_abs_diff'])"
  done
 done
done
