#!/bin/bash
# r6 A/B: k_rows_ws TAIL (loader waves sum half of each block's last unit,
# SMFV_WS_TAIL=1) against the same binary without it and against the build
# before the change (libsmfv_ab.so), alternated on one box; parity first
# (the GPU parity suite's tiled cases with TAIL on).
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"
OUT=$ROOT/gpurun_out/r6_tail; mkdir -p "$OUT"
SMFV_WS_TAIL=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "golden or tiled or cop20k or live or row_pair or narrow or columnwise or permuted" \
    > "$OUT/pytest_tail.log" 2>&1
rc=$?; echo "pytest (TAIL on) rc=$rc"; tail -n 2 "$OUT/pytest_tail.log"; [ $rc -eq 0 ] || exit $rc
A="--no-cpu-baseline --no-vendor --no-rebind --no-copy-floor --no-warm"
for r in 1 2 3; do
  for cfg in cop20k_k32 cop20kirr_k32 cop20k_k128; do
    for v in ab new0 new1; do
      case $v in ab) L=libsmfv_ab.so; T=0;; new0) L=libsmfv.so; T=0;; new1) L=libsmfv.so; T=1;; esac
      SMFV_LIB=$L SMFV_WS_TAIL=$T timeout -k 10 300 python bench.py --config $cfg $A > "$OUT/${cfg}_${v}_$r.json" 2> "$OUT/${cfg}_${v}_$r.log"
      rc=$?; [ $rc -eq 0 ] || { echo "bench $cfg $v rc=$rc"; exit $rc; }
      python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['ms_per_step'], d['check']['ok'])" "$OUT/${cfg}_${v}_$r.json" "$cfg $v $r"
    done
  done
done
