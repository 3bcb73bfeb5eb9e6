#!/bin/bash
# r6: the CLI's first calls on the cop20k surrogate beside the reference's
# own kernels on 16 host ranks (scripts/cli_cop20k.sh), then the NONZERO rank
# plans of the headline at p = 2 / 4 / 8 (one-GPU projections).
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"
OUT=$ROOT/gpurun_out/r6_cli; mkdir -p "$OUT"
SMFV_TIMING=1 timeout -k 10 500 bash scripts/cli_cop20k.sh > "$OUT/cli.log" 2>&1
rc=$?; echo "cli rc=$rc"; grep -E "time|Results" "$OUT/cli.log" | head -30; [ $rc -eq 0 ] || exit $rc
for p in 2 4 8; do
  timeout -k 10 300 python bench.py --config cop20k_k32 --variant NONZERO --rank-plans $p --steps 100 --warmup 10 \
      > "$OUT/nz_p$p.json" 2> "$OUT/nz_p$p.log"
  rc=$?; [ $rc -eq 0 ] || { echo "nz p$p rc=$rc"; exit $rc; }
  python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print('NONZERO p', sys.argv[2], d['rank_local_us_max'], d['rank_local_us_min'], d['check']['ok'])" "$OUT/nz_p$p.json" $p
done
