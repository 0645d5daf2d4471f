#!/bin/bash
# Per-kernel times of library builds on one stream (serialized kernels):
#   LIBS="libmcpt.so libmcpt_base.so" ARGS="" bash scripts/kt_ab.sh
# rocprofv3 kernel-trace stats per build under gpurun_out/kt_ab/<lib>/
set -e
R=$PWD
export TMPDIR=/tmp
for lib in $LIBS; do
  O=$R/gpurun_out/kt_ab/$lib
  mkdir -p $O
  (cd /tmp && MCPT_LIB_PATH=$R/montecarlopathtracer_amd/lib/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats \
     --output-format csv -d $O -o run -- python3 $R/bench.py --no-alt --no-pmc --no-cpu-baseline --steps 1 --warmup 0 \
     --wf-streams 1 $ARGS > $O/log 2>&1)
  python3 - $O <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"]; n = n[n.find("wf_"):n.find("(mcpt::K")] if "wf_" in n else n[:40]
    print(f"  {float(r['TotalDurationNs'])/1e6:9.2f} ms {int(r['Calls']):5d} calls  {n}")
PY
done
