set -e
O=gpurun_out/ab_ws; mkdir -p $O
L=$PWD/montecarlopathtracer_amd/lib
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_edge_scenes.py -k "sorted" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do
for lib in libmcpt_base.so libmcpt.so; do
  for w in c2s c2; do
    a=""; [ $w = c2s ] && a="--wf-sort"
    MCPT_LIB_PATH=$L/$lib timeout -k 10 300 python bench.py --no-alt --steps 5 --warmup 1 --no-cpu-baseline --no-pmc --no-extra $a > $O/b_${lib}_${w}_$r.log 2>&1
    echo "round $r $lib $w: $(grep -o '"value": [0-9.]*' $O/b_${lib}_${w}_$r.log | head -1)"
  done
done
done
