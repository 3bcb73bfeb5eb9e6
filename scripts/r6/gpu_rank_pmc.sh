#!/bin/bash
# r6: HBM bytes per launch of every rank's plan of the p-rank decompositions
# (the roofline.traffic of an N-GPU bench line): for p in
# ${PS:-2 4 8} and each rank r, `bench.py --rank-plans p --rank-only r`
# under rocprofv3, FETCH_SIZE and WRITE_SIZE in passes of their own (kernel
# trace only).  Fold with scripts/r6/pmc_rank_traffic.py.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r6_rankpmc; mkdir -p "$OUT"
CFG=${CFG:-cop20k_k32}
export TMPDIR=/tmp
cd /tmp
for p in ${PS:-2 4 8}; do
  for r in $(seq 0 $((p - 1))); do
    for c in FETCH_SIZE WRITE_SIZE; do
      d="$OUT/${CFG}_p${p}r${r}_$c"
      timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c -d "$d" -o pmc --output-format csv \
        -- python3 "$ROOT/bench.py" --config $CFG --rank-plans $p --rank-only $r --steps 20 --warmup 2 \
        > "$d.log" 2>&1
      rc=$?; echo "p$p r$r $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
    done
  done
done
