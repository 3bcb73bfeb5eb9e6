#!/bin/bash
# r6: per-config bench lines (configs 1, 4, 5 + the headline trio) on the
# round's tree, each followed by a rocprofv3 kernel trace of the same command
# (--stats; medians from the trace by scripts/r6/kernel_trace_summary.py).
# Every GPU step under its own limit; stop at the first failure.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"
TAG=${TAG:-cfg}
OUT=$ROOT/gpurun_out/r6_$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
for spec in ${CONFIGS:-"cop20k_k1:200" "pow10m_k32:100" "syn80m_k32:10"}; do
  c=${spec%%:*}; s=${spec##*:}
  timeout -k 10 400 python bench.py --config $c --steps $s ${BENCH_ARGS:-} > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.log"
  rc=$?; echo "bench $c rc=$rc"; cut -c1-300 "$OUT/bench_$c.json"; [ $rc -eq 0 ] || exit $rc
  if [ -n "${PROF:-1}" ]; then
    (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$c" -o prof --output-format csv \
        -- python3 "$ROOT/bench.py" --config $c --steps $s --no-cpu-baseline --no-warm --no-rebind --no-vendor \
        --no-copy-floor > "$OUT/profbench_$c.json" 2> "$OUT/profbench_$c.log")
    rc=$?; echo "rocprof $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
  fi
done
