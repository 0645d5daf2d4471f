set -e
R=$PWD; O=$R/gpurun_out/ktsur; mkdir -p $O; export TMPDIR=/tmp
for lib in libmcpt.so libmcpt_sur.so; do for sc in scene01 cornell_bunny70k; do
 (cd /tmp && MCPT_LIB_PATH=$R/montecarlopathtracer_amd/lib/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${lib}_$sc -o run -- python3 $R/bench.py --scene $sc --wf-streams 1 --wf-batch 134217728 --no-alt --no-pmc --no-extra --no-cpu-baseline --steps 2 --warmup 1 > $O/${lib}_$sc.log 2>&1)
done; done
echo done
