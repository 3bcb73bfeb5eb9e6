#!/bin/bash
# (r5) What bounds k_rows_wsn (a ColumnWise rank's 4-column window at p = 8):
# kernel-trace stats and PMC passes (one counter group per pass) of
# bench.py --variant COLUMNWISE --rank-plans 8 on the stencil stand-in.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/wsnprof; mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="--config ${CFG:-cop20k_k32} --variant COLUMNWISE --rank-plans 8 --no-cpu-baseline --no-vendor --steps 50 --warmup 5"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o prof --output-format csv \
    -- python3 "$ROOT/bench.py" $ARGS > "$OUT/stats.json" 2> "$OUT/stats.log")
rc=$?; echo "stats rc=$rc"; [ $rc -eq 0 ] || exit $rc
find "$OUT/stats" -name "*kernel_stats.csv" -exec head -n 6 {} \; | cut -c 1-220
for ctr in FETCH_SIZE WRITE_SIZE "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
  tag=$(echo $ctr | cut -d' ' -f1)
  (cd /tmp && timeout -k 10 -s KILL 180 rocprofv3 --kernel-trace --pmc $ctr -d "$OUT/pmc_wsn/$tag" -o pmc --output-format csv \
      -- python3 "$ROOT/bench.py" $ARGS > "$OUT/pmc_$tag.log" 2>&1)
  rc=$?; echo "pmc $tag rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
