#!/bin/bash
# Round-6 second set: the GPU suite on HEAD (sign-ordered child boxes), an A/B
# of the SAH rule's cost constants on the C2 SAH line, and the default bench
# line.  Output under $OUT (default gpurun_out/r06b).
set -e
O=${OUT:-gpurun_out/r06b}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { echo "tests FAILED"; tail -40 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
LIBS="libmcpt.so libmcpt_sah_ci10.so libmcpt_sah_ci12.so libmcpt_sah_ci25.so" ROUNDS=2 STEPS=10 NOTEST=1 NOALT=1 \
  ARGS="--kd-build sah --no-c4" bash scripts/ab2.sh
mkdir -p $O/ab_sah && cp gpurun_out/ab2/b_*.log $O/ab_sah/
timeout -k 10 600 python bench.py > $O/default_bench.jsonl 2> $O/default_bench.err
python3 - $O/default_bench.jsonl <<'PY'
import json, sys
ln = [json.loads(x) for x in open(sys.argv[1]) if x.startswith("{")][-1]
print("C2", ln["value"], ln["ms_per_step"], "frac", ln["roofline"]["frac"])
for k, v in (ln.get("extra_lines") or {}).items():
    print(k, v.get("value"), v.get("ms_per_step"))
PY
