#!/bin/bash
# bench-only A/B of library builds: LIBS="a.so b.so" ARGS="--spp 256" bash scripts/ab_bench.sh
set -e
for round in 1 2; do
for lib in $LIBS; do
  MCPT_LIB_PATH=$PWD/montecarlopathtracer_amd/lib/$lib timeout -k 10 300 python bench.py --pipeline megakernel --steps 2 --warmup 1 --no-cpu-baseline --no-pmc --no-alt $ARGS > gpurun_out/abb.log 2>gpurun_out/abb.err
  echo "round $round $lib: $(grep -o '"value": [0-9.]*' gpurun_out/abb.log) rays/path $(grep -o '"rays_per_path": [0-9.]*' gpurun_out/abb.log) $(grep "phase" gpurun_out/abb.err | head -1)"
done
done
