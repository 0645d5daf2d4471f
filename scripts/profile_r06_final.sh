#!/bin/bash
# Round-6 final records at HEAD (run on the GPU box): smoke(), the driver's
# bench command (20 steps, 5 warmup) with its PMC csv kept, and rocprofv3
# kernel-trace stats of the C2 frame -- default streams and one stream (the
# line's avg_launch_ms agreement).  Output under $OUT (default gpurun_out/r06final).
set -e
R=$PWD
O=${OUT:-gpurun_out/r06final}
mkdir -p $O
O=$(cd $O && pwd)
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -2 $O/smoke.log
timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 --keep-pmc $O/pmc_wf > $O/bench.jsonl 2> $O/bench.err
python3 - $O/bench.jsonl <<'PY'
import json, sys
ln = [json.loads(x) for x in open(sys.argv[1]) if x.startswith("{")][-1]
print("C2", ln["value"], ln["ms_per_step"], "frac", ln["roofline"]["frac"], "avg_launch_ms", ln["roofline"].get("avg_launch_ms"))
for k, v in (ln.get("extra_lines") or {}).items():
    print(k, v.get("value"), v.get("ms_per_step"))
PY
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_c2 -o run -- \
   python3 $R/bench.py --no-alt --no-pmc --no-extra --no-cpu-baseline --steps 2 --warmup 1 > $O/kt_c2.log 2>&1)
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt1_c2 -o run -- \
   python3 $R/bench.py --wf-streams 1 --wf-batch 134217728 --no-alt --no-pmc --no-extra --no-cpu-baseline \
   --steps 2 --warmup 1 > $O/kt1_c2.log 2>&1)
echo traces done
