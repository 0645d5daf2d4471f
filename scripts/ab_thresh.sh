#!/bin/bash
# ready-threshold sweep of the default library: THRESH="24 32 40" bash scripts/ab_thresh.sh
set -e
for round in 1 2; do
for th in $THRESH; do
  MCPT_READY_THRESH=$th timeout -k 10 300 python bench.py --pipeline megakernel --steps 2 --warmup 1 --no-cpu-baseline --no-pmc --no-alt $ARGS > gpurun_out/abt.log 2>gpurun_out/abt.err
  echo "round $round thresh $th: $(grep -o '"value": [0-9.]*' gpurun_out/abt.log)"
done
done
