#!/bin/bash
# Wavefront workspace against throughput: C2 timed at (streams, batch) pairs.
#   PAIRS="3:134217728 2:33554432 3:16777216" bash scripts/mem_curve.sh
set -e
mkdir -p gpurun_out/mem
PAIRS=${PAIRS:-"3:134217728 2:67108864 3:33554432 2:33554432 3:16777216 2:16777216 4:16777216 4:8388608"}
for pr in $PAIRS; do
  s=${pr%%:*}; b=${pr##*:}
  timeout -k 10 300 python bench.py --no-alt --no-pmc --no-cpu-baseline --no-extra --steps ${STEPS:-5} --warmup 1 --wf-streams $s --wf-batch $b $ARGS > gpurun_out/mem/s${s}_b${b}.log 2>&1
  python3 - gpurun_out/mem/s${s}_b${b}.log "$s x $b" <<'PY'
import json, sys
ln = [json.loads(x) for x in open(sys.argv[1]) if x.startswith("{")][-1]
print(f"{sys.argv[2]}: {ln['value']/1e3:.3f} G rays/s  workspace {ln['config']['schedule']['workspace_GB']} GB")
PY
done
