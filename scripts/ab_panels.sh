#!/bin/bash
# A/B of the K > 32 unit order, alternating on one box: OLD (libsmfv_lab.so = a
# copy of the previous product build), NEW serpentine panels (SMFV_WS_PSPLIT=0),
# NEW panel split (SMFV_WS_PSPLIT=1)
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/ab_panels
for cfg in ${CFGS:-cop20k_k128 cop20k_k32}; do
 for r in 1 2; do
  for v in old serp split; do
    case $v in old) E="SMFV_LAB=1";; serp) E="SMFV_WS_PSPLIT=0";; split) E="SMFV_WS_PSPLIT=1";; esac
    env $E timeout -k 10 200 python bench.py --config $cfg --no-cpu-baseline --no-vendor --no-copy-floor --no-rebind \
      > gpurun_out/ab_panels/${cfg}_${v}_$r.json 2> gpurun_out/ab_panels/${cfg}_${v}_$r.log || exit $?
    tail -n 1 gpurun_out/ab_panels/${cfg}_${v}_$r.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg', '$v', round(d['ms_per_step']*1e3, 3), d['roofline']['frac'], d['check']['ok'], d['check']['max_abs_diff'])"
  done
 done
done
