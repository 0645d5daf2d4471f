#!/bin/bash
# wavefront extend-VGPR / shade-size A/B: CFGS="libmcpt.so:0 libmcpt_x.so:1" (lib:shade768)
set -e
for round in 1 2; do
for cfg in $CFGS; do
  lib=${cfg%%:*}; sh=${cfg#*:}
  if [ "$sh" = 1 ]; then export MCPT_WF_SHADE768=1; else unset MCPT_WF_SHADE768; fi
  MCPT_LIB_PATH=$PWD/montecarlopathtracer_amd/lib/$lib timeout -k 10 300 python bench.py --no-alt --no-pmc --no-cpu-baseline --steps 2 --warmup 1 $ARGS > gpurun_out/x.log 2>&1
  echo "round $round $lib shade768=$sh: $(grep -o '"value": [0-9.]*' gpurun_out/x.log)"
done
done
unset MCPT_WF_SHADE768
