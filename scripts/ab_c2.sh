#!/bin/bash
# C2 A/B (round 6): the GPU suite on the working tree's libmcpt.so, then
# interleaved C2 rounds (queue order; megakernel timed beside it) against
# libmcpt_base.so (HEAD).  Output under $OUT (gpurun_out/ab_c2).
set -e
O=${OUT:-gpurun_out/ab_c2}; mkdir -p $O
L=$PWD/montecarlopathtracer_amd/lib
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
for r in $(seq 1 ${ROUNDS:-3}); do
for lib in libmcpt_base.so libmcpt.so; do
  MCPT_LIB_PATH=$L/$lib timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-pmc --no-extra \
    > $O/b_${lib}_$r.log 2>&1
  echo "round $r $lib c2: $(grep -o '"value": [0-9.]*' $O/b_${lib}_$r.log | head -2 | tr '\n' ' ')"
done
done
