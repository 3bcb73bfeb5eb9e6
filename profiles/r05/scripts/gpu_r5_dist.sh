#!/bin/bash
# r5: balanced / chunked distributed plans -- the GPU tests that pin them,
# then the one-GPU rank-plan projections under both partitions and the
# decomposed bench at N = 1 (chunked plan timed beside the value's).
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out/r5dist; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "dist_plan" > "$OUT/pytest_parity_dist.log" 2>&1
rc=$?; echo "pytest parity dist rc=$rc"; tail -n 3 "$OUT/pytest_parity_dist.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_dist_parity.py tests/test_gpu_rank_plans_fullsize.py tests/test_gpu_large_goldens.py \
    > "$OUT/pytest_dist.log" 2>&1
rc=$?; echo "pytest dist rc=$rc"; tail -n 3 "$OUT/pytest_dist.log"; [ $rc -eq 0 ] || exit $rc
for cfg in cop20kirr_k32 cop20k_k32; do
  for part in balanced reference; do
    timeout -k 10 300 python bench.py --config $cfg --rank-plans 8 --partition $part --steps 100 --warmup 10 \
        > "$OUT/rank8_${cfg}_$part.json" 2> "$OUT/rank8_${cfg}_$part.log"
    rc=$?; echo "rank-plans 8 $cfg $part rc=$rc"; cut -c 1-420 "$OUT/rank8_${cfg}_$part.json"; [ $rc -eq 0 ] || exit $rc
  done
done
timeout -k 10 300 python bench.py --config cop20kirr_k32 --rank-plans 8 --rank-chunks 3 --steps 100 --warmup 10 \
    > "$OUT/rank8_cop20kirr_k32_chunks3.json" 2> "$OUT/rank8_cop20kirr_k32_chunks3.log"
rc=$?; echo "rank-plans 8 chunks3 rc=$rc"; cut -c 1-300 "$OUT/rank8_cop20kirr_k32_chunks3.json"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --mode decomposed --no-cpu-baseline --steps 100 --warmup 10 \
    > "$OUT/decomposed_n1.json" 2> "$OUT/decomposed_n1.log"
rc=$?; echo "decomposed N=1 rc=$rc"; cut -c 1-300 "$OUT/decomposed_n1.json"
