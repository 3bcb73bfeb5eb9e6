#!/bin/bash
# r5: FETCH_SIZE / WRITE_SIZE / TCP-TCC requests of the live-values kernel
# against the snapshot kernel (cop20k stand-in, K = 32), one counter group per pass
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r5livepmc; mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
for mode in snap live; do
  [ $mode = live ] && A="--live-values" || A=""
  i=0
  for ctrs in FETCH_SIZE WRITE_SIZE "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_VALU"; do
    i=$((i+1))
    timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $ctrs -d "$OUT/$mode/p$i" -o pmc --output-format csv \
       -- python3 "$ROOT/bench.py" --no-cpu-baseline --no-vendor --no-warm --no-rebind --no-copy-floor --steps 20 --warmup 2 $A \
       > "$OUT/${mode}_p$i.log" 2>&1
    rc=$?; echo "$mode pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
  python3 "$ROOT/scripts/pmc_summary.py" "$OUT/$mode" k_rows_ws > "$OUT/summary_$mode.txt"
  cat "$OUT/summary_$mode.txt"
done
