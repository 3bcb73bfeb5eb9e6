#!/bin/bash
# A/B of the narrow-panel row kernel on the COLUMNWISE rank plans (one-GPU
# projection, bench.py --rank-plans p), alternating on one box: OLD
# (libsmfv_lab.so = a copy of the previous product build) against NEW
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/ab_rank_cw
for cfg in ${CFGS:-cop20k_k32 cop20kirr_k32}; do
 for p in ${PS:-2 4 8}; do
  for v in old new; do
    [ $v = old ] && E="SMFV_LAB=1" || E="SMFV_LAB=0"
    env $E timeout -k 10 300 python bench.py --config $cfg --variant ${VARIANT:-COLUMNWISE} --rank-plans $p \
      > gpurun_out/ab_rank_cw/${cfg}_${p}_${v}.json 2> gpurun_out/ab_rank_cw/${cfg}_${p}_${v}.log || exit $?
    tail -n 1 gpurun_out/ab_rank_cw/${cfg}_${p}_${v}.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg p=$p $v', d['rank_local_us_max'], d['rank_local_us_min'], d.get('check', d.get('checks')))"
  done
 done
done
