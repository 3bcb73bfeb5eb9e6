#!/bin/bash
# PMC passes over a short bench run (one counter group per pass, kernel
# trace only -- never combined with sys/runtime traces).  Stops at the first
# crash/timeout.  Usage: TAG=x PMC_ARGS="--config cop20k_k32" bash scripts/gpu_pmc.sh
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
TAG=${TAG:-pmc}
mkdir -p "$OUT/pmc_$TAG"
export TMPDIR=/tmp
cd /tmp
i=0
# counter groups separated by ';'
SETS=${PMC_SETS:-"FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum;TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum;SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVES"}
IFS=';' read -r -a GROUPS_ARR <<< "$SETS"
for ctrs in "${GROUPS_ARR[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $ctrs -d "$OUT/pmc_$TAG/p$i" -o pmc --output-format csv \
     -- python3 "$ROOT/bench.py" --no-cpu-baseline --steps 20 --warmup 2 ${PMC_ARGS:-} > "$OUT/pmc_$TAG/p$i.log" 2>&1
  rc=$?; echo "pmc pass $i ($ctrs) rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
