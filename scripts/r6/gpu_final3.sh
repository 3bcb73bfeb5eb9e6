#!/bin/bash
# r6 final tree (third pass, after the p = 3 / 5 rank-plan cases): the whole GPU suite, smoke, the default bench (headline with
# cpu_baseline, floor probes, rocSPARSE, warm and rebind legs), then the
# irregular and K = 128 lines and a cold-only kernel trace of each of the
# three.  Every GPU step under its own limit; stop at the first failure.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"
OUT=$ROOT/gpurun_out/r6final3; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q -rs --timeout 300 --timeout-method thread -m gpu tests > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 6 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -n 2 "$OUT/smoke.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.log"
rc=$?; echo "bench rc=$rc"; cut -c 1-300 "$OUT/bench_default.json"; [ $rc -eq 0 ] || exit $rc
for c in cop20kirr_k32 cop20k_k128; do
  timeout -k 10 400 python bench.py --config $c > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.log"
  rc=$?; echo "bench $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
for c in cop20k_k32 cop20kirr_k32 cop20k_k128; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$c" -o prof --output-format csv \
      -- python3 "$ROOT/bench.py" --config $c --no-cpu-baseline --no-warm --no-rebind --no-vendor --no-copy-floor \
      > "$OUT/profbench_$c.json" 2> "$OUT/profbench_$c.log")
  rc=$?; echo "rocprof $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
