#!/bin/bash
# Lane use of the traversal loops (MCPT_PHASE_TIMING builds): one C2 frame per
# library on one stream; the library prints the descent / triangle / burst lane
# use to stderr when its stats are read.
#   LIBS="libmcpt_ph0.so libmcpt_ph1.so" bash scripts/phase_ab.sh
set -e
mkdir -p gpurun_out/phase
for lib in $LIBS; do
  MCPT_LIB_PATH=$PWD/montecarlopathtracer_amd/lib/$lib timeout -k 10 300 python bench.py --no-alt --no-pmc --no-cpu-baseline --no-extra --steps 1 --warmup 0 --wf-streams 1 $ARGS > gpurun_out/phase/$lib.log 2>&1
  echo "$lib: $(grep -h 'lane use' gpurun_out/phase/$lib.log | tail -1)"
done
