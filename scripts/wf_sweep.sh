#!/bin/bash
# wavefront refill-threshold x library sweep (bench only, scene01, 256 spp)
set -e
for lib in $LIBS; do
  for th in $THS; do
    MCPT_LIB_PATH=$PWD/montecarlopathtracer_amd/lib/$lib MCPT_WF_REFILL=$th timeout -k 10 200 python bench.py --pipeline wavefront --spp ${SPP:-256} --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/wfs.log 2>&1
    echo "$lib th=$th $(grep -o '"value": [0-9.]*' gpurun_out/wfs.log)"
  done
done
