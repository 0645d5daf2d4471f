#!/bin/bash
# Sweep one scheduling field: bench.py --set FIELD=V for each V (no PMC, one box).
#   FIELD=wf_refill VALUES="4 8 12" ARGS="--scene cornell_bunny70k" bash scripts/set_sweep.sh
set -e
mkdir -p gpurun_out/sweep
for v in $VALUES; do
  timeout -k 10 300 python bench.py --no-alt --no-pmc --no-cpu-baseline --no-extra --steps ${STEPS:-5} --warmup 1 --set $FIELD=$v $ARGS > gpurun_out/sweep/${FIELD}_$v.log 2>&1
  python3 - gpurun_out/sweep/${FIELD}_$v.log "$FIELD=$v" <<'PY'
import json, sys
ln = [json.loads(x) for x in open(sys.argv[1]) if x.startswith("{")][-1]
print(f"{sys.argv[2]}: {ln['value']/1e3:.3f} G rays/s ({ln['ms_per_step']} ms)")
PY
done
