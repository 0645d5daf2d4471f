#!/bin/bash
# A/B of alternative library builds (MCPT_LIB_PATH) on the wavefront pipeline:
# wavefront parity tests per build, then interleaved C2 (and optionally C4) benches.
#   LIBS="libmcpt.so libmcpt_x.so" ROUNDS=3 ARGS="" bash scripts/ab_wf_libs.sh
set -e
for lib in $LIBS; do
  MCPT_LIB_PATH=$PWD/montecarlopathtracer_amd/lib/$lib timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -m gpu -x -k wavefront > gpurun_out/abwl_tests_$lib.log 2>&1 || { echo "$lib: parity FAILED"; tail -5 gpurun_out/abwl_tests_$lib.log; exit 1; }
  echo "$lib: $(tail -1 gpurun_out/abwl_tests_$lib.log)"
done
for round in $(seq 1 ${ROUNDS:-2}); do
for lib in $LIBS; do
  MCPT_LIB_PATH=$PWD/montecarlopathtracer_amd/lib/$lib timeout -k 10 200 python bench.py --pipeline wavefront --no-alt --steps 3 --warmup 1 --no-cpu-baseline --no-pmc $ARGS > gpurun_out/abwl_$lib.log 2>&1
  echo "round $round $lib: $(grep -o '"value": [0-9.]*' gpurun_out/abwl_$lib.log | head -1)"
done
done
