#!/bin/bash
# parity tests, then bench at several ready thresholds
set -e
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py tests/test_gpu_math.py -q -m gpu -x > gpurun_out/sweep_tests.log 2>&1
for t in ${THRESHS:-1 16 32 48 64}; do
  MCPT_READY_THRESH=$t timeout -k 10 200 python bench.py --pipeline megakernel --no-alt --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/sweep_$t.log 2>&1
  echo "thresh $t: $(grep -o '"value": [0-9.]*' gpurun_out/sweep_$t.log | head -1)"
done
