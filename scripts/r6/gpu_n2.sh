#!/bin/bash
# r6: `bench.py --gpus 2` on a one-GPU box (two ranks started by the bench;
# RCCL refuses two ranks on one device, so the line is the labelled replicas
# fallback) -- it must carry the CPU/MPI baseline.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"
OUT=$ROOT/gpurun_out/r6_n2; mkdir -p "$OUT"
timeout -k 10 600 python bench.py --gpus 2 --steps 50 --warmup 5 > "$OUT/bench_gpus2.json" 2> "$OUT/bench_gpus2.log"
rc=$?; echo "bench --gpus 2 rc=$rc"
python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); c=d.get('cpu_baseline') or {}; print('n_gpus', d.get('n_gpus'), 'fallback', bool(d.get('decomposed_fallback')), 'cpu', c.get('kind'), c.get('value'), c.get('cores'))" "$OUT/bench_gpus2.json"
exit $rc
