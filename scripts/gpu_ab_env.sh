#!/bin/bash
# A/B of lab-build switches: for each "ENV=VAL ..." set in AB_LIST (';'
# separated) run bench.py $AB_ARGS with the lab library (SMFV_LAB=1) and
# those variables; prints ms per step and the check result per set.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
TAG=${TAG:-ab}
IFS=';' read -ra SETS <<< "${AB_LIST:?set AB_LIST}"
for e in "${SETS[@]}"; do
  env SMFV_LAB=1 $e timeout -k 10 ${BENCH_TIMEOUT:-240} python bench.py --no-cpu-baseline --no-vendor ${AB_ARGS:-} \
      > "$OUT/ab_tmp.json" 2>> "$OUT/ab_$TAG.log"
  rc=$?
  if [ $rc -ne 0 ]; then echo "rc=$rc for: $e"; tail -5 "$OUT/ab_$TAG.log"; exit $rc; fi
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); d['_env']=sys.argv[2]; open(sys.argv[3],'a').write(json.dumps(d)+'\n'); print(sys.argv[2], '->', d['ms_per_step']*1e3, 'us', d['roofline']['frac'], 'warm', d['warm']['avg_launch_ms']*1e3, (d.get('check') or {}).get('ok'))" "$OUT/ab_tmp.json" "$e" "$OUT/ab_$TAG.jsonl"
done
