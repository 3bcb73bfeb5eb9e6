#!/bin/bash
# Runs bench.py once per argument set (BENCH_LIST, sets separated by ';'),
# each under its own time limit; one JSON line per set lands in
# gpurun_out/benchlist_$TAG.jsonl (stderr in benchlist_$TAG.log).  Stops at
# the first failure.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
TAG=${TAG:-list}
IFS=';' read -ra SETS <<< "${BENCH_LIST:?set BENCH_LIST}"
for a in "${SETS[@]}"; do
  echo "== $a" | tee -a "$OUT/benchlist_$TAG.log"
  timeout -k 10 ${BENCH_TIMEOUT:-300} python bench.py $a > "$OUT/benchlist_tmp.json" 2>> "$OUT/benchlist_$TAG.log"
  rc=$?
  if [ $rc -ne 0 ]; then echo "rc=$rc for: $a"; tail -5 "$OUT/benchlist_$TAG.log"; exit $rc; fi
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); d['_args']=sys.argv[2]; print(json.dumps(d))" "$OUT/benchlist_tmp.json" "$a" >> "$OUT/benchlist_$TAG.jsonl"
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], '->', d['ms_per_step'], 'ms', r.get('frac'), (d.get('plan') or {}).get('tiles'), (d.get('check') or {}).get('ok'))" "$OUT/benchlist_tmp.json" "$a"
done
