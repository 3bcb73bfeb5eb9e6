#!/bin/bash
# r6: the decomposed (RCCL) bench path at N = 1 -- the code an N-GPU line
# runs (rank-0 CPU baseline before the GPU, distributed plans, per-rank
# roofline with the slowest rank's traffic lookup) -- on a one-GPU box.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"
OUT=$ROOT/gpurun_out/r6_dec1; mkdir -p "$OUT"
timeout -k 10 400 python bench.py --mode decomposed --steps 100 --warmup 10 > "$OUT/bench_decomposed_n1.json" 2> "$OUT/bench_decomposed_n1.log"
rc=$?; echo "bench decomposed N=1 rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/bench_decomposed_n1.log"; exit $rc; }
python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d['roofline']; c=d.get('cpu_baseline') or {}; print(d['n_gpus'], d['ms_per_step'], r['rank'], r['avg_launch_ms'], r['traffic'], r['per_rank'], c.get('kind'), c.get('cores'), c.get('value'), d['check'])" "$OUT/bench_decomposed_n1.json"
