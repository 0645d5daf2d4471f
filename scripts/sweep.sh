#!/bin/bash
# Interleaved sweep of one scheduling field through bench.py --set (GPU box):
#   KEY=wf_refill VALS="8 16 24" ROUNDS=2 ARGS="--scene cornell_bunny70k" bash scripts/sweep.sh
set -e
mkdir -p gpurun_out/sweep
for round in $(seq 1 ${ROUNDS:-2}); do
for v in $VALS; do
  timeout -k 10 300 python bench.py --no-alt --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline --no-pmc --set $KEY=$v $ARGS > gpurun_out/sweep/${KEY}_$v.log 2>&1
  echo "round $round $KEY=$v: $(grep -o '"value": [0-9.]*' gpurun_out/sweep/${KEY}_$v.log | head -1)"
done
done
