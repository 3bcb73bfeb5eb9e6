#!/bin/bash
# Round evidence, in parts (PART=tests|bench|prof|configs|pmc): every step
# has its own time limit and the first failure ends the call.  Outputs in
# gpurun_out/ev_$TAG/ (merged back by gpurun; copy what is judged into
# profiles/rNN/).
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
TAG=${TAG:-r02}
OUT=$ROOT/gpurun_out/ev_$TAG; mkdir -p "$OUT"
run() {  # run <limit> <log> <cmd...>
  local lim=$1 log=$2; shift 2
  echo "== $*" >> "$OUT/steps.log"
  timeout -k 10 "$lim" "$@" > "$OUT/$log" 2>&1
  local rc=$?
  echo "rc=$rc $log" | tee -a "$OUT/steps.log"
  return $rc
}
case "${PART:-tests}" in
tests)
  run 900 pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread || exit $?
  run 300 smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit $?
  ;;
bench)
  run 400 bench_cop20k_k32.json python bench.py || exit $?
  ;;
prof)
  export TMPDIR=/tmp
  (cd /tmp && run 400 prof_cop20k_k32.log rocprofv3 --kernel-trace --stats -d "$OUT/prof_cop20k_k32" -o prof \
      --output-format csv -- python3 "$ROOT/bench.py" --no-cpu-baseline --steps 200 --warmup 20) || exit $?
  ;;
configs)
  CONFIGS=${CONFIGS:-cop20k_k128 cop20k_k1 pow10m_k32 pow10m_k1 cop20k_perm_k32}
  for c in $CONFIGS; do
    run 400 bench_$c.json python bench.py --config $c --no-cpu-baseline || exit $?
  done
  for v in COLUMNWISE NONZERO; do
    run 300 bench_cop20k_k32_$v.json python bench.py --variant $v --no-cpu-baseline --no-vendor || exit $?
  done
  run 300 bench_cop20k_k32_decomposed_n1.json python bench.py --mode decomposed --no-cpu-baseline || exit $?
  run 300 bench_cop20k_k128_mfma.json python bench.py --config cop20k_k128 --mfma --no-cpu-baseline --no-vendor || exit $?
  run 300 bench_cop20k_k32_mfma.json python bench.py --mfma --no-cpu-baseline --no-vendor || exit $?
  ;;
syn80m)
  run 900 bench_syn80m_k32.json python bench.py --config syn80m_k32 --steps 10 --warmup 2 || exit $?
  ;;
cli)
  # the reference CLI's path on the surrogate under rocprofv3: shows which
  # kernels sparseMatrixFatVectorMultiply* run (k_rows_ws through the plan cache)
  run 120 write_mtx.log python -c "import sparsematrixmultiplicationmpi_amd as s; s.writeMatrixMarketFile('/tmp/cop20k_surrogate.mtx', s.cop20k_surrogate(), symmetric=True)" || exit $?
  export TMPDIR=/tmp
  (cd /tmp && run 300 cli_prof.log rocprofv3 --kernel-trace --stats -d "$OUT/prof_cli" -o prof --output-format csv \
      -- "$ROOT/sparsematrixmultiplicationmpi_amd/smfv_main" 32 /tmp/cop20k_surrogate.mtx) || exit $?
  ;;
ablate)
  ABL_LIST=${ABL_LIST:-SMFV_WS_ABL=0 SMFV_WS_ABL=1 SMFV_WS_ABL=2 SMFV_WS_ABL=3 SMFV_WS_ABL=0}
  for e in $ABL_LIST; do
    run 240 abl_$e.json env SMFV_LAB=1 $e python bench.py --no-cpu-baseline --no-vendor --no-check || exit $?
  done
  ;;
pmc)
  export TMPDIR=/tmp
  for cfg in ${PMC_CONFIGS:-cop20k_k32 pow10m_k32}; do
    i=0
    for ctrs in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
      i=$((i+1))
      (cd /tmp && run 300 pmc_${cfg}_p$i.log rocprofv3 --kernel-trace --pmc $ctrs -d "$OUT/pmc_$cfg/p$i" -o pmc \
          --output-format csv -- python3 "$ROOT/bench.py" --config $cfg --no-cpu-baseline --no-vendor --steps 20 --warmup 2) || exit $?
    done
  done
  ;;
esac
