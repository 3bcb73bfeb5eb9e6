mkdir -p gpurun_out
export SMFV_LAB=1
SMFV_K1_PIPE=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "k1 or k_sweep or spmv" > gpurun_out/r3_k1pipe_tests.log 2>&1; rc=$?; echo tests=$rc; tail -n 4 gpurun_out/r3_k1pipe_tests.log; [ $rc -le 1 ] || exit $rc
for bpc in 0 1 2 4 8 0 2 4; do
  SMFV_K1_PIPE=$bpc timeout -k 10 200 python bench.py --config cop20k_k1 --no-cpu-baseline --no-vendor > gpurun_out/r3_k1_bpc$bpc.log 2>&1 || exit 3
  python -c "import json,sys; d=json.loads(open('gpurun_out/r3_k1_bpc$bpc.log').read().strip().splitlines()[-1]); print('bpc $bpc', d['ms_per_step']*1000, 'us', d['roofline']['frac'], d['check']['ok'], d['warm']['avg_launch_ms']*1000)"
done
