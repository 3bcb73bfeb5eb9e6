#!/bin/bash
# A/B of bench.py argument sets: for each set in AB_LIST (';' separated) run
# bench.py --no-cpu-baseline --no-vendor <set> with the product library;
# prints ms per step, roofline fraction and the check per set.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
TAG=${TAG:-abargs}
IFS=';' read -ra SETS <<< "${AB_LIST:?set AB_LIST}"
for a in "${SETS[@]}"; do
  timeout -k 10 ${BENCH_TIMEOUT:-240} python bench.py --no-cpu-baseline --no-vendor $a \
      > "$OUT/ab_tmp.json" 2>> "$OUT/ab_$TAG.log"
  rc=$?
  if [ $rc -ne 0 ]; then echo "rc=$rc for: $a"; tail -5 "$OUT/ab_$TAG.log"; exit $rc; fi
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); d['_args']=sys.argv[2]; open(sys.argv[3],'a').write(json.dumps(d)+'\n'); print(sys.argv[2], '->', round(d['ms_per_step']*1e3,2), 'us', d['roofline']['frac'], 'warm', round(d['warm']['avg_launch_ms']*1e3,2), 'tiles', d['plan']['tiles'], 'parts', d['plan'].get('xcd_parts'), (d.get('check') or {}).get('ok'))" "$OUT/ab_tmp.json" "$a" "$OUT/ab_$TAG.jsonl"
done
