#!/bin/bash
# Full GPU session: tests + smoke + bench + rocprof stats + PMC traffic +
# a 2-rank rehearsal of the N>1 bench path (both ranks on the one GPU).
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
TAG=${TAG:-round}
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 600 python -m pytest tests -m gpu -x -q > "$OUT/pytest_$TAG.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 4 "$OUT/pytest_$TAG.log"; ok $rc || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -n 2 "$OUT/smoke_$TAG.log"; ok $rc || exit $rc
timeout -k 10 400 python bench.py > "$OUT/bench_$TAG.log" 2>&1
rc=$?; echo "bench rc=$rc"; tail -n 1 "$OUT/bench_$TAG.log"; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$TAG" -o prof --output-format csv \
    -- python3 "$ROOT/bench.py" --no-cpu-baseline --steps 200 --warmup 20 > "$OUT/profbench_$TAG.log" 2>&1)
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
find "$OUT/prof_$TAG" -name "*kernel_stats.csv" -exec head -n 4 {} \;
PMC_SETS="FETCH_SIZE;WRITE_SIZE" TAG=$TAG bash scripts/gpu_pmc.sh; rc=$?; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29531 bench.py --gpus 2 --steps 50 --warmup 5 > "$OUT/bench2_$TAG.log" 2>&1
rc=$?; echo "bench N=2 rehearsal rc=$rc"; tail -n 1 "$OUT/bench2_$TAG.log"
