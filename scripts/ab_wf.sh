#!/bin/bash
# A/B of wavefront library builds: the full GPU suite on the first (product)
# build, then interleaved C2 (and optional extra-args) bench rounds per build.
#   LIBS="libmcpt.so libmcpt_x.so" ROUNDS=2 ARGS="" bash scripts/ab_wf.sh
set -e
mkdir -p gpurun_out/ab
first=${LIBS%% *}
if [ -z "$NOTEST" ]; then
  MCPT_LIB_PATH=$PWD/montecarlopathtracer_amd/lib/$first timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab/tests.log 2>&1 || { echo "tests FAILED"; tail -30 gpurun_out/ab/tests.log; exit 1; }
  tail -1 gpurun_out/ab/tests.log
fi
for round in $(seq 1 ${ROUNDS:-2}); do
for lib in $LIBS; do
  MCPT_LIB_PATH=$PWD/montecarlopathtracer_amd/lib/$lib timeout -k 10 300 python bench.py --no-alt --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline --no-pmc --no-c5 $ARGS > gpurun_out/ab/b_$lib.log 2>&1
  echo "round $round $lib: $(grep -o '"value": [0-9.]*' gpurun_out/ab/b_$lib.log | head -1) $(grep -o '"kernel_ms_avg": [0-9.]*' gpurun_out/ab/b_$lib.log)"
done
done
