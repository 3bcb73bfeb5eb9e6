#!/bin/bash
# One GPU session: parity tests -> smoke -> bench -> rocprofv3 kernel stats.
# Every GPU step has its own time limit; a crash/timeout (rc not 0/1) ends
# the session.  Outputs land in gpurun_out/ (merged back by gpurun).
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
TAG=${TAG:-run}
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }

if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > "$OUT/pytest_gpu_$TAG.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -n 25 "$OUT/pytest_gpu_$TAG.log"
  ok $rc || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -n 5 "$OUT/smoke_$TAG.log"
  ok $rc || exit $rc
fi
timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py ${BENCH_ARGS:-} > "$OUT/bench_$TAG.log" 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 4000 "$OUT/bench_$TAG.log"
[ $rc -eq 0 ] || exit $rc
if [ "${SKIP_PROF:-0}" != 1 ]; then
  export TMPDIR=/tmp
  (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$TAG" -o prof --output-format csv \
      -- python3 "$ROOT/bench.py" --no-cpu-baseline --steps 100 --warmup 10 ${BENCH_ARGS:-} > "$OUT/prof_$TAG.log" 2>&1)
  rc=$?; echo "rocprof rc=$rc"
  find "$OUT/prof_$TAG" -name "*kernel_stats.csv" -exec head -n 12 {} \;
fi
