#!/bin/bash
# r5 session 3 final tree: GPU suite, smoke, default bench, the ColumnWise
# rank-plan projections on the rounds-picked k_rows_wsn plans (both stand-ins,
# p = 8 / 4), then rocprofv3 kernel stats + FETCH/WRITE PMC of the p = 8
# stencil projection.  Every GPU step under its own limit; stop at the first failure.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out/r5final2; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -n 2 "$OUT/smoke.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.log"
rc=$?; echo "bench rc=$rc"; cut -c 1-300 "$OUT/bench_default.json"; [ $rc -eq 0 ] || exit $rc
for cfg in cop20k_k32 cop20kirr_k32; do
  for p in 8 4; do
    timeout -k 10 300 python bench.py --config $cfg --variant COLUMNWISE --rank-plans $p --steps 100 --warmup 10 \
        > "$OUT/cw_${cfg}_p$p.json" 2> "$OUT/cw_${cfg}_p$p.log" || exit $?
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['rank_local_us_max'], d['rank_local_us_min'], d['check']['ok'], d['ranks'][0]['tiles'])" "$OUT/cw_${cfg}_p$p.json" "$cfg p$p"
  done
done
ARGS="--config cop20k_k32 --variant COLUMNWISE --rank-plans 8 --no-cpu-baseline --no-vendor --steps 50 --warmup 5"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/wsn_stats" -o prof --output-format csv \
    -- python3 "$ROOT/bench.py" $ARGS > "$OUT/wsn_stats.json" 2> "$OUT/wsn_stats.log")
rc=$?; echo "stats rc=$rc"; [ $rc -eq 0 ] || exit $rc
find "$OUT/wsn_stats" -name "*kernel_stats.csv" -exec head -n 6 {} \; | cut -c 1-220
for ctr in FETCH_SIZE WRITE_SIZE; do
  (cd /tmp && timeout -k 10 -s KILL 180 rocprofv3 --kernel-trace --pmc $ctr -d "$OUT/wsn_pmc/$ctr" -o pmc --output-format csv \
      -- python3 "$ROOT/bench.py" $ARGS > "$OUT/wsn_pmc_$ctr.log" 2>&1)
  rc=$?; echo "pmc $ctr rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
