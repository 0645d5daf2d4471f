#!/bin/bash
# GPU suite on the product build, then interleaved C4 bench rounds per library
# build, then the product build's C4 PMC passes (kept csv).
#   LIBS="libmcpt.so libmcpt_x.so" ROUNDS=2 [NOTEST=1] OUT=gpurun_out/abc4 bash scripts/ab_c4.sh
set -e
O=${OUT:-gpurun_out/abc4}
mkdir -p $O
first=${LIBS%% *}
if [ -z "$NOTEST" ]; then
  MCPT_LIB_PATH=$PWD/montecarlopathtracer_amd/lib/$first timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests FAILED"; tail -40 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
for round in $(seq 1 ${ROUNDS:-2}); do
for lib in $LIBS; do
  MCPT_LIB_PATH=$PWD/montecarlopathtracer_amd/lib/$lib timeout -k 10 300 python bench.py --scene cornell_bunny70k --no-alt --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline --no-pmc $ARGS > $O/b_${lib}_$round.log 2>&1
  python3 - $O/b_${lib}_$round.log "$round $lib" <<'PY'
import json, sys
ln = [json.loads(x) for x in open(sys.argv[1]) if x.startswith("{")][-1]
print(f"{sys.argv[2]}: c4 {ln['value']/1e3:.3f} G rays/s ({ln['kernel_ms_avg']} ms)")
PY
done
done
if [ -z "$NOPMC" ]; then
  timeout -k 10 400 python bench.py --scene cornell_bunny70k --no-alt --steps 1 --warmup 1 --no-cpu-baseline --keep-pmc $O/pmc > $O/pmc_line.jsonl 2> $O/pmc_line.err
  python3 - $O/pmc_line.jsonl <<'PY'
import json, sys
ln = [json.loads(x) for x in open(sys.argv[1]) if x.startswith("{")][-1]
r = ln["roofline"]; k = r["pipeline"]["kernels"]["extend"]
print("extend read", k["hbm_read_GB"], "write", k["hbm_write_GB"], "ms", k["ms"], "split", r.get("read_split"))
PY
fi
