#!/bin/bash
# r5: the --gpus N launcher on the one-GPU box (both ranks on device 0: RCCL
# refuses a duplicated device, so the line must say n_gpus 2 with a labelled
# decomposed_fallback) + the headline bench without the CPU leg.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out/r5; mkdir -p "$OUT"
timeout -k 10 300 python bench.py --gpus 2 --steps 50 --warmup 5 --no-vendor --no-copy-floor --no-rebind \
    > "$OUT/bench_gpus2.json" 2> "$OUT/bench_gpus2.log"
rc=$?; echo "bench --gpus 2 rc=$rc"; cut -c 1-600 "$OUT/bench_gpus2.json"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench_default.json" 2> "$OUT/bench_default.log"
rc=$?; echo "bench rc=$rc"; cut -c 1-400 "$OUT/bench_default.json"
