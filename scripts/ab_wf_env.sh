#!/bin/bash
# bench-only A/B of environment settings on the wavefront pipeline:
#   ENVS="MCPT_WF_REFILL=12 MCPT_WF_REFILL=16" ARGS="--scene cornell_bunny70k --spp 512" ROUNDS=2 bash scripts/ab_wf_env.sh
# (each entry of ENVS is one setting, or several joined by commas)
set -e
for round in $(seq 1 ${ROUNDS:-2}); do
for ev in $ENVS; do
  env ${ev//,/ } timeout -k 10 300 python bench.py --pipeline wavefront --no-alt --steps 3 --warmup 1 --no-cpu-baseline --no-pmc $ARGS > gpurun_out/abwe.log 2>gpurun_out/abwe.err
  echo "round $round $ev: $(grep -o '"value": [0-9.]*' gpurun_out/abwe.log)"
done
done
