#!/bin/bash
# GPU suite + the default bench line (with its PMC csv kept) on one box.
#   OUT=gpurun_out/r05 [BENCH_ARGS=...] [NOTEST=1] bash scripts/gpu_check.sh
set -e
O=${OUT:-gpurun_out/check}
mkdir -p $O
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { echo "tests FAILED"; tail -40 $O/gputest.log; exit 1; }
  tail -1 $O/gputest.log
fi
timeout -k 10 600 python bench.py --steps ${STEPS:-10} --warmup 2 --keep-pmc $O/pmc_wf $BENCH_ARGS > $O/bench.jsonl 2> $O/bench.err
python3 - $O/bench.jsonl <<'PY'
import json, sys
ln = [json.loads(x) for x in open(sys.argv[1]) if x.startswith("{")][-1]
r = ln["roofline"]
print(f"C2 {ln['value']/1e3:.3f} G rays/s {ln['ms_per_step']} ms  hbm frac {r.get('frac')}  valu {r.get('valu', {}).get('useful_lane_frac')}")
alt = ln.get("other_pipeline") or {}
print(f"megakernel {alt.get('value', 0)/1e3:.3f}")
for k, v in (ln.get("extra_lines") or {}).items():
    if "value" in v:
        print(f"{k} {v['value']/1e3:.3f} G rays/s {v['ms_per_step']} ms  hbm frac {v['roofline'].get('frac')}")
    else:
        print(k, v)
PY
