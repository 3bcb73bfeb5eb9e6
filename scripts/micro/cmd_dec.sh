timeout -k 10 240 python bench.py --mode decomposed --no-cpu-baseline --no-vendor > gpurun_out/bench_dec1.json 2>gpurun_out/bench_dec1.log || { tail -5 gpurun_out/bench_dec1.log; exit 1; }
tail -c 1500 gpurun_out/bench_dec1.json
bash scripts/micro/cmd_n2.sh | tail -c 600
