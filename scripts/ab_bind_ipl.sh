#!/bin/bash
# A/B of the bind kernel's items per lane (SMFV_BIND_IPL), alternating on one box:
# plan.rebind_each_step's bind_ms (bind alone, in the graph) and bind + execute
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/bind_ipl
for cfg in ${CFGS:-cop20k_k32 cop20kirr_k32}; do
 for r in 1 2; do
  for ipl in 1 2 4 8; do
    SMFV_BIND_IPL=$ipl timeout -k 10 200 python bench.py --config $cfg --no-cpu-baseline --no-vendor --no-copy-floor \
      > gpurun_out/bind_ipl/${cfg}_${ipl}_$r.json 2> gpurun_out/bind_ipl/${cfg}_${ipl}_$r.log || exit $?
    tail -n 1 gpurun_out/bind_ipl/${cfg}_${ipl}_$r.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); rb=d['plan']['rebind_each_step']; print('$cfg ipl=$ipl', round(d['ms_per_step']*1e3,2), 'bind', round(rb['bind_ms']*1e3,2), 'b+e', round(rb['bind_plus_execute_ms']*1e3,2), d['check']['ok'], rb.get('check'))"
  done
 done
done
