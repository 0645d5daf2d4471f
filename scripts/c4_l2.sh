#!/bin/bash
# L2 hit rate and time of the C4 extend per library build (one C4 frame under a
# TCC_HIT / TCC_MISS pass; kernels serialized by the PMC pass).
#   LIBS="libmcpt_x0.so libmcpt_x1.so" bash scripts/c4_l2.sh
set -e
R=$PWD
export TMPDIR=/tmp
mkdir -p $R/gpurun_out/c4_l2
for lib in $LIBS; do
  O=$R/gpurun_out/c4_l2/$lib
  rm -rf $O; mkdir -p $O
  (cd /tmp && MCPT_LIB_PATH=$R/montecarlopathtracer_amd/lib/$lib timeout -k 10 240 rocprofv3 --pmc TCC_HIT TCC_MISS \
     --output-format csv -d $O -o run -- python3 $R/bench.py --scene cornell_bunny70k --no-alt --no-pmc --no-extra \
     --no-cpu-baseline --steps 1 --warmup 0 $ARGS > $O/log 2>&1)
  python3 - $O $lib <<'PY'
import importlib.util, os, sys
spec = importlib.util.spec_from_file_location("b", os.path.join(os.getcwd(), "bench.py"))
b = importlib.util.module_from_spec(spec); spec.loader.exec_module(b)
k = b.read_wf_kernels(sys.argv[1])
e = k.get("extend", {})
h, m = e.get("TCC_HIT", 0.0), e.get("TCC_MISS", 0.0)
print(f"{sys.argv[2]}: extend {e.get('ns', 0)/1e6:.1f} ms over {e.get('dispatches')} dispatches, "
      f"L2 hit {h/max(h+m,1):.4f} ({h/1e9:.2f} G hits, {m/1e9:.2f} G misses)")
PY
done
