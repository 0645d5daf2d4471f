#!/bin/bash
# A/B: parity tests + bench for alternative library builds (MCPT_LIB_PATH), interleaved
set -e
for lib in $LIBS; do
  MCPT_LIB_PATH=$PWD/montecarlopathtracer_amd/lib/$lib timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -m gpu -x > gpurun_out/ab_tests_$lib.log 2>&1 || { echo "$lib: parity FAILED"; tail -5 gpurun_out/ab_tests_$lib.log; }
done
for round in 1 2; do
for lib in $LIBS; do
  MCPT_LIB_PATH=$PWD/montecarlopathtracer_amd/lib/$lib timeout -k 10 200 python bench.py --pipeline megakernel --no-alt --steps 2 --warmup 1 --no-cpu-baseline --no-pmc > gpurun_out/ab_$lib.log 2>&1
  echo "round $round $lib: $(grep -o '"value": [0-9.]*' gpurun_out/ab_$lib.log | head -1) $(grep -o '"stack_spills_per_ray": [0-9.]*' gpurun_out/ab_$lib.log)"
done
done
