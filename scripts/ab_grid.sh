#!/bin/bash
# library x ready-threshold grid: LIBS="a.so b.so" THRESH="28 32" bash scripts/ab_grid.sh
set -e
for round in 1 2; do
for lib in $LIBS; do
for th in $THRESH; do
  MCPT_LIB_PATH=$PWD/montecarlopathtracer_amd/lib/$lib MCPT_READY_THRESH=$th timeout -k 10 300 python bench.py --pipeline megakernel --no-alt --steps 2 --warmup 1 --no-cpu-baseline --no-pmc $ARGS > gpurun_out/abg.log 2>gpurun_out/abg.err
  echo "round $round $lib thresh $th: $(grep -o '"value": [0-9.]*' gpurun_out/abg.log)"
done
done
done
