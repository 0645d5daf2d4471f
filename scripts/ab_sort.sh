#!/bin/bash
# Round 6: the material sort moved into the shade (per-block LDS counting sort)
# -- the GPU suite on the working tree's libmcpt.so, then interleaved rounds of
# C2 queue order, C2 sorted and C4 against the previous build (libmcpt_lists.so:
# HEAD before the change, class-list sort).  Output under $OUT (gpurun_out/sortab).
set -e
O=${OUT:-gpurun_out/sortab}; mkdir -p $O
L=$PWD/montecarlopathtracer_amd/lib
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
B="--no-alt --steps 5 --warmup 1 --no-cpu-baseline --no-pmc --no-extra"
for r in $(seq 1 ${ROUNDS:-3}); do
for lib in libmcpt_lists.so libmcpt.so; do
  for w in c2 c2s c4; do
    a=""; [ $w = c2s ] && a="--wf-sort"; [ $w = c4 ] && a="--scene cornell_bunny70k"
    MCPT_LIB_PATH=$L/$lib timeout -k 10 300 python bench.py $B $a > $O/b_${lib}_$w.log 2>&1
    echo "round $r $lib $w: $(grep -o '"value": [0-9.]*' $O/b_${lib}_$w.log | head -1)"
  done
done
done
