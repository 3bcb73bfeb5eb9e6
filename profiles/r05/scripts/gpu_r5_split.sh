#!/bin/bash
# (r5) SPLIT: the loader waves of k_rows_ws sum the other 16 columns of each
# panel once their DMAs are out (k_rows_ws_split, SMFV_WS_SPLIT=1).  Parity
# of the tiled kernels with SPLIT on, then an A/B on one box, alternating per
# config: this build (split off: the refactored k_rows_ws), split on, and the
# previous build (libsmfv_ab.so).
# (Kept as the record of that run: the split kernel was measured 12-18 % slower and
# never committed, profiles/r05/wsn/README.md; without it both legs run k_rows_ws.)
cd ${GRAFT_REPO_ROOT:-$(pwd)}
out=gpurun_out/split
mkdir -p $out
if [ -z "${SKIP_TESTS:-}" ]; then
  SMFV_WS_SPLIT=1 timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
      -k "${TESTS:-row_pair or tiled_plan_bitwise or every_row_length or golden or full_size or k_sweep or k128 or permuted}" \
      > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
  tail -2 $out/pytest.log
fi
for cfg in ${CFGS:-cop20k_k128 cop20k_k32 cop20kirr_k32}; do
  for r in $(seq 1 ${ROUNDS:-2}); do
    for leg in ${LEGS:-split new old}; do
      case $leg in
        new) L=libsmfv.so; S=0 ;;
        split) L=libsmfv.so; S=1 ;;
        old) L=libsmfv_ab.so; S=0 ;;
      esac
      SMFV_WS_SPLIT=$S SMFV_LIB=$L timeout -k 10 200 python bench.py --config $cfg --no-cpu-baseline --no-vendor --no-copy-floor \
          --no-rebind ${EXTRA:-} > $out/${cfg}_${leg}_$r.json 2> $out/${cfg}_${leg}_$r.log || exit $?
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('$cfg', '$leg', round(d['ms_per_step']*1e3, 3), d['roofline']['frac'], d['plan']['tiles'], d['check']['ok'])" $out/${cfg}_${leg}_$r.json
    done
  done
done
