#!/bin/bash
# wavefront stream/batch sweep: CFGS="2:134217728 4:67108864" ARGS="..." ROUNDS=3 bash scripts/ab_wf_cfg.sh
set -e
for round in $(seq 1 ${ROUNDS:-2}); do
for c in $CFGS; do
  n=${c%%:*}; b=${c#*:}
  MCPT_WF_STREAMS=$n timeout -k 10 300 python bench.py --pipeline wavefront --wf-batch $b --steps 2 --warmup 1 --no-cpu-baseline --no-pmc --no-alt $ARGS > gpurun_out/abw.log 2>gpurun_out/abw.err
  echo "round $round streams $n batch $b: $(grep -o '"value": [0-9.]*' gpurun_out/abw.log)"
done
done
