#!/bin/bash
# per-kernel time of the wavefront pipeline for libraries in LIBS (C2 and C4):
#   LIBS="a.so b.so" bash scripts/wf_kstats.sh   (run on the GPU box)
set -e
export TMPDIR=/tmp
R=$PWD
for lib in $LIBS; do
  for cfg in "c2:" "c4:--scene cornell_bunny70k --spp 256"; do
    name=${cfg%%:*}; args=${cfg#*:}
    D=$R/gpurun_out/wfk_${lib%.so}_$name
    MCPT_LIB_PATH=$R/montecarlopathtracer_amd/lib/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 $R/bench.py --pipeline wavefront --steps 1 --warmup 0 --no-cpu-baseline --no-pmc $args > $D.jsonl 2> $D.err
    echo "$lib $name: $(grep -o '"value": [0-9.]*' $D.jsonl)"
    python3 - "$D/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "wf_" in r["Name"]:
        print("   %-14s %8.1f ms total (%s calls)" % (r["Name"].split("wf_")[1].split("(")[0].split("<")[0], float(r["TotalDurationNs"]) / 2e6, r["Calls"]))
PY
  done
done
