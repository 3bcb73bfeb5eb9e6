#!/bin/bash
# A/B of the lab k_rows_ws with LDS-counter handshakes (SMFV_WS_ABL=9)
# against the product kernel (SMFV_WS_ABL=0) on the cop20k surrogate, K=32.
mkdir -p gpurun_out
export SMFV_LAB=1
SMFV_WS_ABL=9 timeout -k 10 120 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 60 --timeout-method thread -k "tiled_plan_bitwise or every_row_length or tiny or cop20k_surrogate_full" > gpurun_out/r3_abl9_tests.log 2>&1; rc=$?; echo tests=$rc; tail -n 4 gpurun_out/r3_abl9_tests.log; [ $rc -le 1 ] || exit $rc
for i in 1 2 3; do
  for abl in 0 9; do
    SMFV_WS_ABL=$abl timeout -k 10 120 python bench.py --no-cpu-baseline --no-vendor ${EXTRA:-} > gpurun_out/r3_abl${abl}_$i.log 2>&1 || exit 3
    python -c "import json; d=json.loads(open('gpurun_out/r3_abl${abl}_$i.log').read().strip().splitlines()[-1]); print('abl $abl', round(d['ms_per_step']*1000,3), 'us warm', round(d['warm']['avg_launch_ms']*1000,3), d['check']['ok'])"
  done
done
