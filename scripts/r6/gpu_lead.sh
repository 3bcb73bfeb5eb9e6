#!/bin/bash
# r6 A/B: live-values plans with lead pads (16-byte aligned value pairs,
# the default) against the r5 layout (SMFV_LIVE_NO_LEAD=1), same binary:
# the GPU parity file first, then execute-only live timing alternated.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"
OUT=$ROOT/gpurun_out/r6_lead; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    > "$OUT/pytest_parity.log" 2>&1
rc=$?; echo "pytest parity rc=$rc"; tail -n 2 "$OUT/pytest_parity.log"; [ $rc -eq 0 ] || exit $rc
A="--no-cpu-baseline --no-vendor --no-rebind --no-copy-floor --no-warm --live-values"
for r in 1 2 3; do
  for cfg in cop20k_k32 cop20kirr_k32 cop20k_k128; do
    for v in lead nolead; do
      if [ $v = nolead ]; then export SMFV_LIVE_NO_LEAD=1; else unset SMFV_LIVE_NO_LEAD; fi
      timeout -k 10 300 python bench.py --config $cfg $A > "$OUT/${cfg}_${v}_$r.json" 2> "$OUT/${cfg}_${v}_$r.log"
      rc=$?; [ $rc -eq 0 ] || { echo "bench $cfg $v rc=$rc"; exit $rc; }
      python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['ms_per_step'], d['check']['ok'], d['plan']['live_values'], d['plan']['tiles'])" "$OUT/${cfg}_${v}_$r.json" "$cfg $v $r"
    done
  done
done
unset SMFV_LIVE_NO_LEAD
