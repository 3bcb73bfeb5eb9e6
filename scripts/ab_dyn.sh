#!/bin/bash
# k_rows_ws tile queue (DYN, the product default) vs the fixed stride
# (SMFV_WS_DYN=0, lab build), alternating on one box, every run checked.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
for cfg in ${CFGS:-cop20k_k32 cop20kirr_k32 cop20k_k128}; do
  AB_ARGS="--config $cfg --no-copy-floor" TAG=dyn_$cfg \
    AB_LIST="SMFV_WS_DYN=1;SMFV_WS_DYN=0;SMFV_WS_DYN=1;SMFV_WS_DYN=0" bash scripts/gpu_ab_env.sh || exit $?
done
