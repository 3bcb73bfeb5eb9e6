#!/bin/bash
# (r4) one-GPU projection of the p-rank decomposition: every rank's share
# timed through its rank plan (bench.py --rank-plans p), per config / variant /
# tiled-kernel geometry; one JSON line each into gpurun_out/rank_plans_$TAG.jsonl
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
TAG=${TAG:-rp}
for cfg in ${CFGS:-cop20k_k32}; do
 for v in ${VARIANTS:-ROWWISE}; do
  for p in ${PS:-2 4 8}; do
   for tk in ${TKS:-auto}; do
    timeout -k 10 ${BENCH_TIMEOUT:-300} python bench.py --config $cfg --variant $v --rank-plans $p \
        --tiled-kernel $tk --steps ${STEPS:-100} ${EXTRA:-} >> "$OUT/rank_plans_$TAG.jsonl" 2>> "$OUT/rank_plans_$TAG.log"
    rc=$?
    if [ $rc -ne 0 ]; then echo "rc=$rc for $cfg $v $p $tk"; tail -5 "$OUT/rank_plans_$TAG.log"; exit $rc; fi
    tail -n 1 "$OUT/rank_plans_$TAG.jsonl" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg', '$v', 'p=%d'%d['p'], '$tk', 'max %.2f us min %.2f us' % (d['rank_local_us_max'], d['rank_local_us_min']), 'xbytes', d['exchange_bytes_max'], 'tiles', [r['tiles'] for r in d['ranks']], 'ok', d['check']['ok'])"
   done
  done
 done
done
