set -e
R=$PWD
export TMPDIR=/tmp
for lib in ${LIBS:-libmcpt.so}; do
cd /tmp
MCPT_LIB_PATH=$R/montecarlopathtracer_amd/lib/$lib timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/kt_c4_$lib -o run -- python3 $R/bench.py --scene cornell_bunny70k --no-pmc --no-cpu-baseline --no-alt --steps 1 --warmup 0 --wf-streams 1 > $R/gpurun_out/kt_c4_$lib.log 2>&1
cd $R
echo "== $lib $(grep -o '"value": [0-9.]*' gpurun_out/kt_c4_$lib.log)"
python3 scripts/wf_bounce_times.py gpurun_out/kt_c4_$lib
done
