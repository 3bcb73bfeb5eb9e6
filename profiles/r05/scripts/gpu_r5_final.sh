#!/bin/bash
# r5 final tree: the whole GPU suite, smoke, the default bench (headline
# config with its cpu_baseline, rocSPARSE, warm, rebind legs).  Every GPU step
# under its own limit; stop at the first failure.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out/r5final; mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -n 2 "$OUT/smoke.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.log"
rc=$?; echo "bench rc=$rc"; cut -c 1-400 "$OUT/bench_default.json"; [ $rc -eq 0 ] || exit $rc
