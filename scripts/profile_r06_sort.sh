#!/bin/bash
# Where the material-sorted wavefront frame goes (round 6): the C2 frame
# (1024^2 x 1024 spp) with wf_sort = 1 against queue order, kernel traces on
# one stream so the per-kernel sums add up to the frame.  Output under $OUT
# (default gpurun_out/r06sort).
set -e
R=$PWD
O=${OUT:-gpurun_out/r06sort}
mkdir -p $O
O=$(cd $O && pwd)
export TMPDIR=/tmp
for v in queue sorted; do
  f=""; [ $v = sorted ] && f="--wf-sort"
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt1_$v -o run -- \
     python3 $R/bench.py $f --wf-streams 1 --wf-batch 134217728 --no-alt --no-pmc --no-extra --no-cpu-baseline \
     --steps 1 --warmup 1 > $O/kt1_$v.log 2>&1)
  timeout -k 10 300 python3 bench.py $f --no-alt --no-pmc --no-extra --no-cpu-baseline --steps 3 --warmup 1 \
     > $O/bench_$v.jsonl 2> $O/bench_$v.err
done
python3 - $O <<'PY'
import csv, glob, json, sys
o = sys.argv[1]
for v in ("queue", "sorted"):
    ln = [json.loads(x) for x in open(f"{o}/bench_{v}.jsonl") if x.startswith("{")][-1]
    print(v, "G rays/s", ln["value"] / 1e3, "ms", ln["ms_per_step"])
    f = glob.glob(f"{o}/kt1_{v}/**/run_kernel_stats.csv", recursive=True)
    for row in sorted(csv.DictReader(open(f[0])), key=lambda r: -float(r["TotalDurationNs"]))[:8]:
        print(f"  {row['Name'][:60]:60s} calls {row['Calls']:>5s} total {float(row['TotalDurationNs'])/1e6:9.1f} ms"
              f" avg {float(row['AverageNs'])/1e6:7.3f}")
PY
