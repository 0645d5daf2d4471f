#!/bin/bash
# Round-5 profile set at HEAD (run on the GPU box via gpurun): the GPU suite and
# the default bench line with its PMC csv (scripts/gpu_check.sh), rocprofv3
# kernel-trace stats of the C2 and C4 wavefront frames (default streams, and one
# stream for the avg_launch_ms agreement), and one rank's C2 share
# at N = 2 / 4 / 8.  Output under gpurun_out/r05final/.
set -e
R=$PWD
O=$R/gpurun_out/r05final
export OUT=$O TMPDIR=/tmp
bash scripts/gpu_check.sh
for sc in scene01 cornell_bunny70k; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$sc -o run -- \
     python3 $R/bench.py --scene $sc --no-alt --no-pmc --no-extra --no-cpu-baseline --steps 2 --warmup 1 > $O/kt_$sc.log 2>&1)
done
echo profiles done
# the same frames on one stream (kernels one at a time, as in the PMC passes):
# the extend's average launch here is what the bench line's avg_launch_ms times
for sc in scene01 cornell_bunny70k; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt1_$sc -o run -- \
     python3 $R/bench.py --scene $sc --wf-streams 1 --wf-batch 134217728 --no-alt --no-pmc --no-extra --no-cpu-baseline \
     --steps 2 --warmup 1 > $O/kt1_$sc.log 2>&1)
done
echo serial profiles done
timeout -k 10 300 python3 scripts/shard_probe.py 2 4 8 --combos 0:0 > $O/shard_probe.txt 2>&1
grep "N=" $O/shard_probe.txt
