#!/bin/bash
# Round-6 third set: the GPU suite on HEAD (SAH rule with clipped-triangle
# boxes), the SAH-line A/B (perfect splits Ct 2 / 2.5 / 1.5 against the
# previous unclipped rule), then the default bench line.  Output under $OUT.
set -e
O=${OUT:-gpurun_out/r06c}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { echo "tests FAILED"; tail -40 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
rm -rf gpurun_out/ab2
LIBS="libmcpt.so libmcpt_sah_np.so libmcpt_sah_p25.so libmcpt_sah_p15.so" ROUNDS=2 STEPS=10 NOTEST=1 NOALT=1 \
  ARGS="--kd-build sah --no-c4" bash scripts/ab2.sh
mkdir -p $O/ab_sah && cp gpurun_out/ab2/b_*.log $O/ab_sah/
timeout -k 10 600 python bench.py > $O/default_bench.jsonl 2> $O/default_bench.err
python3 - $O/default_bench.jsonl <<'PY'
import json, sys
ln = [json.loads(x) for x in open(sys.argv[1]) if x.startswith("{")][-1]
print("C2", ln["value"], ln["ms_per_step"], "frac", ln["roofline"]["frac"])
for k, v in (ln.get("extra_lines") or {}).items():
    print(k, v.get("value"), v.get("ms_per_step"), (v.get("roofline") or {}).get("valu", {}).get("wave_instr_per_ray"))
PY
