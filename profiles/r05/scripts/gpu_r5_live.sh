#!/bin/bash
# r5: live values (SMFV_PLAN_LIVE_VALUES) -- parity, then the headline configs
# with and without it, alternating on one box (bind + execute leg included).
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out/r5live; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "live or golden or tiled or narrow or cop20k" > "$OUT/pytest_live.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 "$OUT/pytest_live.log"; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for cfg in cop20k_k32 cop20kirr_k32 cop20k_k128; do
    for mode in snap live; do
      [ $mode = live ] && A="--live-values" || A=""
      timeout -k 10 200 python bench.py --config $cfg --no-cpu-baseline --no-vendor --no-copy-floor $A \
          > "$OUT/${cfg}_${mode}_$r.json" 2> "$OUT/${cfg}_${mode}_$r.log" || exit $?
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); rb=d['plan']['rebind_each_step'] or {}; print(sys.argv[2], round(d['ms_per_step']*1e3,3), d['roofline']['frac'], d['check']['ok'], 'bind+exec', round(rb.get('bind_plus_execute_ms',0)*1e3,3), 'bind', round(rb.get('bind_ms',0)*1e3,3))" "$OUT/${cfg}_${mode}_$r.json" "$cfg $mode"
    done
  done
done
