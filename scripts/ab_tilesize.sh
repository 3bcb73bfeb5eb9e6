#!/bin/bash
# Lab: what a unit costs.  Tiles capped at fewer rows (more, smaller units)
# with the lab build's SMFV_WS_MAXROWS; cold bench, alternating on one box.
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
for cfg in cop20k_k32 cop20kirr_k32; do
 for r in 1 2; do
  for rows in 64 56 48 40 32; do
    SMFV_LAB=1 SMFV_WS_MAXROWS=$rows timeout -k 10 200 python bench.py --config $cfg --no-cpu-baseline --no-vendor --no-copy-floor --no-warm > gpurun_out/ts_${cfg}_${rows}_$r.log 2>&1 || exit $?
    tail -n 1 gpurun_out/ts_${cfg}_${rows}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'config':'$cfg','maxrows':$rows,'rep':$r,'tiles':d['plan']['tiles'],'us':round(d['ms_per_step']*1e3,3),'bit_exact':d['check']['max_abs_diff']==0}))"
  done
 done
done
