#!/bin/bash
# K = 1 on the cop20k surrogate: the chunk plan (k_spmv_chunks, 1,024- and
# 2,048-entry chunks via the lab build's SMFV_K1_CHUNK) against the untiled
# k_spmv_stream (--tiles off), in alternation; parity tests first.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "k1 or spmv or k_sweep or golden or degenerate or huge_row" > gpurun_out/r3_k1_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 3 gpurun_out/r3_k1_tests.log; [ $rc -eq 0 ] || exit $rc
for i in $(seq 1 ${ROUNDS:-3}); do
 for cfg in ${CFGS:-cop20k_k1 cop20kirr_k1}; do
  for mode in ${MODES:-off 1024 2048}; do
    if [ $mode = off ]; then args="--tiles off"; env=""; else args=""; env="SMFV_LAB=1 SMFV_K1_CHUNK=$mode"; fi
    env $env timeout -k 10 120 python bench.py --config $cfg --no-cpu-baseline --no-vendor $args > gpurun_out/r3_k1_${cfg}_${mode}_$i.log 2>&1 || exit 3
    python -c "import json; d=json.loads(open('gpurun_out/r3_k1_${cfg}_${mode}_$i.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$cfg $mode', round(d['ms_per_step']*1000,3), 'us', r['kernel'], 'frac', r['frac'], 'copy', (r.get('size_matched_copy') or {}).get('avg_launch_ms'), d['check']['ok'], d['plan']['tiled'], d['plan']['tiles'])"
  done
 done
done
