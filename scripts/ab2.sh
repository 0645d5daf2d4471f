#!/bin/bash
# A/B of library builds on one box: optional GPU suite on the first build, then
# interleaved bench rounds per build (wavefront line + the megakernel beside it).
#   LIBS="libmcpt.so libmcpt_x.so" ROUNDS=2 ARGS="" [NOTEST=1] [NOALT=1] bash scripts/ab2.sh
set -e
mkdir -p gpurun_out/ab2
first=${LIBS%% *}
if [ -z "$NOTEST" ]; then
  MCPT_LIB_PATH=$PWD/montecarlopathtracer_amd/lib/$first timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab2/tests.log 2>&1 || { echo "tests FAILED"; tail -40 gpurun_out/ab2/tests.log; exit 1; }
  tail -1 gpurun_out/ab2/tests.log
fi
alt="--no-alt"; [ -z "$NOALT" ] && alt=""
for round in $(seq 1 ${ROUNDS:-2}); do
for lib in $LIBS; do
  MCPT_LIB_PATH=$PWD/montecarlopathtracer_amd/lib/$lib timeout -k 10 300 python bench.py $alt --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline --no-pmc --no-c5 $ARGS > gpurun_out/ab2/b_${lib}_$round.log 2>&1
  python3 - gpurun_out/ab2/b_${lib}_$round.log "$round $lib" <<'PY'
import json, sys
ln = [json.loads(x) for x in open(sys.argv[1]) if x.startswith("{")][-1]
alt = ln.get("other_pipeline") or {}
c4 = (ln.get("extra_lines") or {}).get("c4") or {}
print(f"{sys.argv[2]}: wf {ln['value']/1e3:.3f} G rays/s ({ln['kernel_ms_avg']} ms)  mk {alt.get('value', 0)/1e3:.3f} ({alt.get('kernel_ms_avg')})"
      + (f"  c4 {c4['value']/1e3:.3f}" if "value" in c4 else ""))
PY
done
done
