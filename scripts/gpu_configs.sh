#!/bin/bash
# Bench lines of the non-headline BASELINE configs + rocprof kernel stats of
# the headline one.  Stops at the first failure.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"
OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; TAG=${TAG:-cfg}
for c in ${CONFIGS:-cop20k_k128 pow10m_k32}; do
  timeout -k 10 300 python bench.py --config $c ${BENCH_ARGS:---no-cpu-baseline} > "$OUT/bench_${c}_$TAG.log" 2>&1
  rc=$?; echo "bench $c rc=$rc"; tail -n 1 "$OUT/bench_${c}_$TAG.log" | cut -c1-300; [ $rc -eq 0 ] || exit $rc
done
if [ -n "${PROF:-1}" ]; then
  export TMPDIR=/tmp
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$TAG" -o prof --output-format csv \
      -- python3 "$ROOT/bench.py" --no-cpu-baseline --steps 200 --warmup 20 > "$OUT/profbench_$TAG.log" 2>&1)
  rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
  find "$OUT/prof_$TAG" -name "*kernel_stats.csv" -exec head -n 4 {} \;
fi
