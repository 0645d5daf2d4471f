#!/bin/bash
# A/B: seed table (TEA-16 pre-pass) vs in-kernel seeding; VARIANTS="lib:ENV=val ..."
set -e
for round in 1 2; do
for v in $VARIANTS; do
  lib=${v%%:*}; ev=${v#*:}
  env $ev MCPT_LIB_PATH=$PWD/montecarlopathtracer_amd/lib/$lib timeout -k 10 300 python bench.py --pipeline megakernel --no-alt --steps 2 --warmup 1 --no-cpu-baseline --no-pmc > gpurun_out/abs.log 2>gpurun_out/abs.err
  echo "round $round $v: $(grep -o '"value": [0-9.]*' gpurun_out/abs.log) $(grep -o '"kernel_ms_avg": [0-9.]*' gpurun_out/abs.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abs.log)"
done
done
