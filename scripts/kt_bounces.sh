set -e
R=$PWD
export TMPDIR=/tmp
for lib in libmcpt.so libmcpt_nopk.so; do
cd /tmp
MCPT_LIB_PATH=$R/montecarlopathtracer_amd/lib/$lib timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/kt_$lib -o run -- python3 $R/bench.py --no-pmc --no-cpu-baseline --no-alt --steps 1 --warmup 0 --wf-streams 1 > $R/gpurun_out/kt_$lib.log 2>&1
cd $R
python3 scripts/wf_bounce_times.py gpurun_out/kt_$lib
done
