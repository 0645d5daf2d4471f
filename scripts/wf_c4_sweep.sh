#!/bin/bash
set -e
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu -x -k "wavefront" > gpurun_out/wf_parity.log 2>&1
for gsh in 6 8 10 12; do
  MCPT_WF_GROUP_SHIFT=$gsh timeout -k 10 300 python bench.py --pipeline wavefront --scene cornell_bunny70k --spp 64 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/wfc4.log 2>&1
  echo "gs=$gsh $(grep -o '"value": [0-9.]*' gpurun_out/wfc4.log)"
done
