#!/bin/bash
# (r4) narrow tiled window: GPU tests first, then the ColumnWise rank plans
# (bench.py --rank-plans p) with the tiled narrow window (default) against
# the untiled row kernel (--tiles off), alternating on one box
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/ab_narrow
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "narrow or tiled_plan_bitwise" > gpurun_out/ab_narrow/pytest_narrow.log 2>&1
rc=$?; tail -n 3 gpurun_out/ab_narrow/pytest_narrow.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_rank_plans_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k COLUMNWISE > gpurun_out/ab_narrow/pytest_rank_cw.log 2>&1
rc=$?; tail -n 3 gpurun_out/ab_narrow/pytest_rank_cw.log; [ $rc -eq 0 ] || exit $rc
for cfg in cop20k_k32 cop20kirr_k32; do
 for p in 2 4 8; do
  for t in auto off; do
    timeout -k 10 300 python bench.py --config $cfg --variant COLUMNWISE --rank-plans $p --tiles $t \
      > gpurun_out/ab_narrow/${cfg}_${p}_$t.json 2> gpurun_out/ab_narrow/${cfg}_${p}_$t.log || exit $?
    tail -n 1 gpurun_out/ab_narrow/${cfg}_${p}_$t.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg p=$p tiles=$t', d['rank_local_us_max'], d['rank_local_us_min'], d['check']['ok'], d['check']['max_abs_diff'])"
  done
 done
done
