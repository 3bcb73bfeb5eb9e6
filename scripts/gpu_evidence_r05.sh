#!/bin/bash
# Round-5 evidence (same recipe as r4) (each GPU step under its own limit; a crash or timeout
# ends the script):
#  1. the headline bench JSON (full default run incl. cpu_baseline) -> bench_$cfg.json
#  2. cold-only rocprofv3 kernel stats of the same config (no warm leg, no
#     rocSPARSE leg): the SpMM, the bind kernels and the copy floor
#  3. FETCH_SIZE / WRITE_SIZE passes (one counter per pass) and the
#     wave-state counters SQ_WAVE_CYCLES / SQ_WAIT_ANY / SQ_WAIT_INST_ANY /
#     SQ_ACTIVE_INST_ANY / SQ_ACTIVE_INST_VALU / SQ_ACTIVE_INST_LDS / SQ_BUSY_CYCLES
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r5ev
mkdir -p "$OUT"
export TMPDIR=/tmp
for cfg in ${CFGS:-cop20k_k32}; do
  if [ -z "$SKIP_BENCH" ]; then
    timeout -k 10 400 python3 "$ROOT/bench.py" --config $cfg ${BENCH_ARGS:-} > "$OUT/bench_$cfg.json" 2> "$OUT/bench_$cfg.log"
    rc=$?; echo "bench $cfg rc=$rc"; [ $rc -eq 0 ] || exit $rc
    cut -c 1-300 "$OUT/bench_$cfg.json"
  fi
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$cfg" -o prof --output-format csv \
      -- python3 "$ROOT/bench.py" --config $cfg --no-cpu-baseline --no-vendor --no-warm --no-rebind --steps 200 --warmup 20 \
      > "$OUT/prof_$cfg.json" 2> "$OUT/prof_$cfg.log")
  rc=$?; echo "rocprof $cfg rc=$rc"; [ $rc -eq 0 ] || exit $rc
  find "$OUT/prof_$cfg" -name "*kernel_stats.csv" -exec head -n 8 {} \; | cut -c 1-200
  [ -n "$NO_PMC" ] && continue
  for ctr in FETCH_SIZE WRITE_SIZE "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES"; do
    tag=$(echo $ctr | cut -d' ' -f1)
    (cd /tmp && timeout -k 10 -s KILL 180 rocprofv3 --kernel-trace --pmc $ctr -d "$OUT/pmc_$cfg/$tag" -o pmc --output-format csv \
        -- python3 "$ROOT/bench.py" --config $cfg --no-cpu-baseline --no-vendor --no-warm --no-rebind --steps 20 --warmup 2 \
        > "$OUT/pmc_${cfg}_$tag.log" 2>&1)
    rc=$?; echo "pmc $cfg $tag rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
