#!/bin/bash
# lab A/B of the narrow row kernel's gathers in flight (SMFV_ROW_CFG=TEAM,H,U)
# on the COLUMNWISE rank plans, alternating on one box
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/ab_row_u
for cfg in ${CFGS:-cop20k_k32 cop20kirr_k32}; do
 for p in 2 4 8; do
  case $p in 2) T=8;; 4) T=4;; 8) T=2;; esac
  for u in 8 16; do
    SMFV_LAB=1 SMFV_ROW_CFG=$T,1,$u timeout -k 10 300 python bench.py --config $cfg --variant COLUMNWISE --rank-plans $p \
      > gpurun_out/ab_row_u/${cfg}_${p}_u$u.json 2> gpurun_out/ab_row_u/${cfg}_${p}_u$u.log || exit $?
    tail -n 1 gpurun_out/ab_row_u/${cfg}_${p}_u$u.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg p=$p T=$T U=$u', d['rank_local_us_max'], d['rank_local_us_min'], d['check']['ok'], d['check']['max_abs_diff'])"
  done
 done
done
