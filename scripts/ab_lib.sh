#!/bin/bash
# A/B of two builds of the same sources, alternating on one box:
#   NEW = libsmfv.so (this tree), OLD = libsmfv_ab.so (a copy of the build to
#   compare against, placed in the package directory before the gpurun call;
#   loaded with SMFV_LIB=libsmfv_ab.so).  CFGS / ROUNDS / EXTRA select what runs;
#   LIBS the libraries and their order within a round (an A/A run: copy the
#   same build to a second name).
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/ab
for cfg in ${CFGS:-cop20k_k32 cop20k_k128 cop20kirr_k32}; do
 for r in $(seq 1 ${ROUNDS:-2}); do
  for lib in ${LIBS:-libsmfv.so libsmfv_ab.so}; do
    SMFV_LIB=$lib timeout -k 10 200 python bench.py --config $cfg --no-cpu-baseline --no-vendor --no-copy-floor \
        --no-rebind ${EXTRA:-} > gpurun_out/ab/ab_${cfg}_${lib%.so}_$r.json 2> gpurun_out/ab/ab_${cfg}_${lib%.so}_$r.log || exit $?
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('$cfg', '$lib', round(d['ms_per_step']*1e3, 3), d['roofline']['frac'], d['check']['ok'], d['check'].get('max_abs_diff'))" gpurun_out/ab/ab_${cfg}_${lib%.so}_$r.json
  done
 done
done
