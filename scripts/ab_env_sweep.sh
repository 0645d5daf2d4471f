#!/bin/bash
# sweep one environment variable of the default library:
#   VAR=MCPT_WF_REFILL VALS="8 16 32" ARGS="--pipeline wavefront" bash scripts/ab_env_sweep.sh
set -e
for round in 1 2; do
for v in $VALS; do
  env $VAR=$v timeout -k 10 300 python bench.py --pipeline megakernel --steps 2 --warmup 1 --no-cpu-baseline --no-pmc --no-alt $ARGS > gpurun_out/abe.log 2>gpurun_out/abe.err
  echo "round $round $VAR=$v: $(grep -o '"value": [0-9.]*' gpurun_out/abe.log)"
done
done
