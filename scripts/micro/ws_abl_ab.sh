#!/bin/bash
# A/B of lab k_rows_ws variants (SMFV_WS_ABL=<n>, libsmfv_lab.so) against the
# product kernel (0) on the cop20k surrogate, K=32, in alternation.  The
# variants that compute a result are checked first by the bitwise tests.
#   ABLS="0 9 10 11"  ROUNDS=3  EXTRA="--fma"
mkdir -p gpurun_out
export SMFV_LAB=1
for abl in ${ABLS:-0 9 10 11}; do
  [ "$abl" = 0 ] && continue
  SMFV_WS_ABL=$abl timeout -k 10 120 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 60 --timeout-method thread -k "tiled_plan_bitwise or every_row_length or tiny or cop20k_surrogate_full" > gpurun_out/r3_abl${abl}_tests.log 2>&1; rc=$?; echo "abl $abl tests=$rc"; tail -n 2 gpurun_out/r3_abl${abl}_tests.log; [ $rc -le 1 ] || exit $rc
done
for i in $(seq 1 ${ROUNDS:-3}); do
  for abl in ${ABLS:-0 9 10 11}; do
    SMFV_WS_ABL=$abl timeout -k 10 120 python bench.py --no-cpu-baseline --no-vendor ${EXTRA:-} > gpurun_out/r3_ab_abl${abl}_$i.log 2>&1 || exit 3
    python -c "import json; d=json.loads(open('gpurun_out/r3_ab_abl${abl}_$i.log').read().strip().splitlines()[-1]); print('abl $abl', round(d['ms_per_step']*1000,3), 'us warm', round(d['warm']['avg_launch_ms']*1000,3), d['check']['ok'], 'copy', (d['roofline'].get('size_matched_copy') or {}).get('avg_launch_ms'))"
  done
done
