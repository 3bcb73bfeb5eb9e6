#!/bin/bash
# (r5) Row pairs: the parity tests that run the tiled kernels, then an A/B on
# one box -- new build (automatic choice), the same build with pairs forced
# on / off (the plan effect alone), and the previous build (libsmfv_ab.so:
# the kernel change) -- alternating, per config.
cd ${GRAFT_REPO_ROOT:-$(pwd)}
out=gpurun_out/pairs
mkdir -p $out
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
      -k "${TESTS:-row_pair or tiled_plan or narrow or live_values or golden}" > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
  tail -2 $out/pytest.log
fi
for cfg in ${CFGS:-cop20kirr_k32 cop20k_k32 cop20k_k128}; do
  for r in $(seq 1 ${ROUNDS:-2}); do
    for leg in ${LEGS:-new single old}; do
      case $leg in
        new) L=libsmfv.so; E="" ;;
        pairs) L=libsmfv.so; E="--row-pairs on" ;;
        single) L=libsmfv.so; E="--row-pairs off" ;;
        old) L=libsmfv_ab.so; E="" ;;
        ws3) L=libsmfv.so; E="--tiled-kernel ws3" ;;
        ws3old) L=libsmfv_ab.so; E="--tiled-kernel ws3" ;;
      esac
      SMFV_LIB=$L timeout -k 10 200 python bench.py --config $cfg --no-cpu-baseline --no-vendor --no-copy-floor \
          --no-rebind $E ${EXTRA:-} > $out/${cfg}_${leg}_$r.json 2> $out/${cfg}_${leg}_$r.log || exit $?
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('$cfg', '$leg', round(d['ms_per_step']*1e3, 3), d['roofline']['frac'], d['plan']['tiles'], d['plan'].get('paired_rows'), d['check']['ok'])" $out/${cfg}_${leg}_$r.json
    done
  done
done
