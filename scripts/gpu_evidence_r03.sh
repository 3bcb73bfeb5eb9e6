#!/bin/bash
# Round-3 evidence: cold-only rocprofv3 kernel stats of the headline (no warm
# leg, no rocSPARSE leg in the same process), FETCH_SIZE / WRITE_SIZE passes
# for the headline and the irregular surrogate.  Each GPU step has its own
# limit; a crash or timeout ends the script.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
for cfg in ${CFGS:-cop20k_k32 cop20kirr_k32}; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/r3prof_$cfg" -o prof --output-format csv \
      -- python3 "$ROOT/bench.py" --config $cfg --no-cpu-baseline --no-vendor --no-warm --steps 200 --warmup 20 \
      > "$OUT/r3prof_$cfg.log" 2>&1)
  rc=$?; echo "rocprof $cfg rc=$rc"; [ $rc -eq 0 ] || exit $rc
  tail -n 1 "$OUT/r3prof_$cfg.log" | cut -c 1-400
  find "$OUT/r3prof_$cfg" -name "*kernel_stats.csv" -exec head -n 4 {} \;
  for ctr in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && timeout -k 10 -s KILL 180 rocprofv3 --kernel-trace --pmc $ctr -d "$OUT/r3pmc_$cfg/$ctr" -o pmc --output-format csv \
        -- python3 "$ROOT/bench.py" --config $cfg --no-cpu-baseline --no-vendor --no-warm --steps 20 --warmup 2 \
        > "$OUT/r3pmc_${cfg}_$ctr.log" 2>&1)
    rc=$?; echo "pmc $cfg $ctr rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
