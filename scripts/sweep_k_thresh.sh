#!/bin/bash
# descent cap (library builds) x ready threshold (env) sweep, bench only
set -e
for lib in $LIBS; do
  for t in $THRESHS; do
    MCPT_LIB_PATH=$PWD/montecarlopathtracer_amd/lib/$lib MCPT_READY_THRESH=$t timeout -k 10 200 python bench.py --pipeline megakernel --no-alt --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/skt.log 2>&1
    echo "$lib thresh $t: $(grep -o '"value": [0-9.]*' gpurun_out/skt.log | head -1)"
  done
done
