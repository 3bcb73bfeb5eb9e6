#!/bin/bash
# which first copy absorbs the runtime's one-time H2D start (h2d_reg_probe.cpp):
# order letter (p / t / g: 4 KiB, huge pages or registered first), warm-up MiB, r = registered warm-up
mkdir -p gpurun_out
for args in "p 0" "g 0" "t 1" "t 8" "t 64" "p 1 r" "p 8 r"; do
  echo "== $args"
  timeout -k 10 60 ./scripts/micro/h2d_reg_probe $args > gpurun_out/h2d_probe.txt || exit 1
  head -n 5 gpurun_out/h2d_probe.txt | grep -v small_copy
done
