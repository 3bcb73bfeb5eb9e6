#!/bin/bash
# (r5) K = 128 (config 3) with the opt-in FMA plan flag (one fused multiply-add
# per term: within the reference's 1e-6, not bit-identical) against the
# default (separate multiply and add, bit-exact), alternating on one box.
cd ${GRAFT_REPO_ROOT:-$(pwd)}
out=gpurun_out/fma128; mkdir -p $out
for r in 1 2 3; do
  for leg in exact fma; do
    E=""; [ $leg = fma ] && E="--fma"
    timeout -k 10 200 python bench.py --config cop20k_k128 --no-cpu-baseline --no-vendor --no-copy-floor --no-rebind $E \
        > $out/k128_${leg}_$r.json 2> $out/k128_${leg}_$r.log || exit $?
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('k128', '$leg', round(d['ms_per_step']*1e3, 3), d['roofline']['frac'], d['check'])" $out/k128_${leg}_$r.json
  done
done
