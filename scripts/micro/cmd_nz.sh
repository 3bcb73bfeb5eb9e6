# GPU suite + NONZERO bench lines (tiled by default on cop20k; --tiles off = merge path)
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_nz.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_nz.log; [ $rc -eq 0 ] || exit $rc
for a in "--variant NONZERO" "--variant NONZERO --tiles off"; do
  timeout -k 10 240 python bench.py --no-cpu-baseline --no-vendor $a > gpurun_out/nz_tmp.json 2>>gpurun_out/nz.log || exit 1
  tail -1 gpurun_out/nz_tmp.json >> gpurun_out/bench_nz.jsonl
  python3 -c "import json; d=json.loads(open('gpurun_out/nz_tmp.json').read().strip().splitlines()[-1]); print('$a', d['ms_per_step']*1e3, d['roofline']['kernel'], d['roofline']['frac'], d['check'])"
done
