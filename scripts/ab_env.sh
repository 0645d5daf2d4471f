#!/bin/bash
# bench-only A/B of environment settings on one library:
#   ENVS="MCPT_TREELET=0 MCPT_TREELET=1" ARGS="--scene cornell_bunny70k --spp 256" bash scripts/ab_env.sh
set -e
for round in 1 2; do
for ev in $ENVS; do
  env $ev timeout -k 10 300 python bench.py --pipeline megakernel --no-alt --steps 2 --warmup 1 --no-cpu-baseline --no-pmc $ARGS > gpurun_out/abe.log 2>gpurun_out/abe.err
  echo "round $round $ev: $(grep -o '"value": [0-9.]*' gpurun_out/abe.log) variant $(grep -o '"kernel_variant": [0-9]*' gpurun_out/abe.log)"
done
done
