#!/bin/bash
# r6: the default bench line (headline + its new mix_matched_copy floor
# probes), then K = 128 on this tree against the r4 build (SMFV_LIB, the
# r4 sources of commit 4cff953 built in-tree), alternated.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"
OUT=$ROOT/gpurun_out/r6_probe; mkdir -p "$OUT"
timeout -k 10 400 python bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.log"
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
python - "$OUT/bench_default.json" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d["roofline"]
print("ms", d["ms_per_step"], "frac", r["frac"], "copy", r["size_matched_copy"]["avg_launch_ms"])
print("mix", json.dumps(r["mix_matched_copy"]))
print("lds", r["lds_staged_bytes_per_launch"])
PY
A="--no-cpu-baseline --no-vendor --no-rebind --no-copy-floor --no-warm"
for i in 1 2; do
  for lib in libsmfv.so libsmfv_r4.so; do
    SMFV_LIB=$lib timeout -k 10 300 python bench.py --config cop20k_k128 $A > "$OUT/k128_${lib}_$i.json" 2> "$OUT/k128_${lib}_$i.log"
    rc=$?; echo "k128 $lib $i rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$OUT/k128_${lib}_$i.json" | head -1)"; [ $rc -eq 0 ] || exit $rc
  done
done
