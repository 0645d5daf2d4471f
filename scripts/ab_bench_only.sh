#!/bin/bash
# bench-only A/B of library builds (no parity: for timing experiments that change the image)
set -e
for round in 1 2; do
for lib in $LIBS; do
  MCPT_LIB_PATH=$PWD/montecarlopathtracer_amd/lib/$lib timeout -k 10 200 python bench.py --pipeline megakernel --no-alt --steps 2 --warmup 1 --no-cpu-baseline $ARGS > gpurun_out/abo_$lib.log 2>&1
  echo "round $round $lib: $(grep -o '"value": [0-9.]*' gpurun_out/abo_$lib.log | head -1)"
done
done
