# L2 (TCC) hit rate of the C4 wavefront extend for library builds (one PMC pass each)
set -e
R=$PWD
export TMPDIR=/tmp
for lib in ${LIBS:-libmcpt.so}; do
cd /tmp
MCPT_LIB_PATH=$R/montecarlopathtracer_amd/lib/$lib timeout -s KILL 200 rocprofv3 --pmc TCC_HIT TCC_MISS TCP_TOTAL_CACHE_ACCESSES TCP_TCC_READ_REQ --output-format csv -d $R/gpurun_out/pmc_c4_$lib -o run -- python3 $R/bench.py --scene cornell_bunny70k --no-pmc --no-cpu-baseline --no-alt --steps 1 --warmup 0 --wf-streams 1 > $R/gpurun_out/pmc_c4_$lib.log 2>&1
cd $R
python3 - $lib <<'PY'
import csv, glob, sys, collections
lib = sys.argv[1]
acc = collections.Counter()
for f in glob.glob(f"gpurun_out/pmc_c4_{lib}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "wf_extend" in r["Kernel_Name"]:
            acc[r["Counter_Name"]] += float(r["Counter_Value"])
h, m = acc["TCC_HIT"], acc["TCC_MISS"]
print(lib, {k: round(v / 1e9, 3) for k, v in acc.items()}, "L2 hit", round(h / (h + m), 4),
      "L1 miss->L2 req / L1 access", round(acc["TCP_TCC_READ_REQ"] / max(acc["TCP_TOTAL_CACHE_ACCESSES"], 1), 4))
PY
done
