# timing-only: the full kernel with 1/3 or 1/2 of the X pieces not staged (results wrong; --no-check)
cd sparsematrixmultiplicationmpi_amd
for v in base skip3 skip2 base skip3 skip2; do
  if [ $v = base ]; then L=0; else cp libsmfv_$v.so libsmfv_lab.so; L=1; fi
  (cd .. && SMFV_LAB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-vendor --no-check > gpurun_out/skip_tmp.json 2>>gpurun_out/skip.log) || exit 1
  python3 -c "import json,sys; d=json.loads(open('../gpurun_out/skip_tmp.json').read().strip().splitlines()[-1]); print(sys.argv[1], round(d['ms_per_step']*1e3,2), 'us warm', round(d['warm']['avg_launch_ms']*1e3,2))" $v
done
