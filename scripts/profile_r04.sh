#!/bin/bash
# Round-4 profile set (run on the GPU box via gpurun): the default bench line
# with its raw PMC csv kept (C2 + the C4 child), then rocprofv3 kernel-trace
# stats of the C2 and C4 wavefront frames.  Output under gpurun_out/r04/.
set -e
R=$PWD
O=$R/gpurun_out/r04
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 bench.py --keep-pmc $O/pmc_wf > $O/bench.jsonl 2> $O/bench.err
tail -c 300 $O/bench.jsonl
for sc in scene01 cornell_bunny70k; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$sc -o run -- \
     python3 $R/bench.py --scene $sc --no-alt --no-pmc --no-extra --no-cpu-baseline --steps 2 --warmup 1 > $O/kt_$sc.log 2>&1)
done
echo profiles done
# the same frames on one stream (kernels one at a time, as in the PMC passes):
# the extend's average launch here is what the bench line's avg_launch_ms times
for sc in scene01 cornell_bunny70k; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt1_$sc -o run -- \
     python3 $R/bench.py --scene $sc --wf-streams 1 --wf-batch 134217728 --no-alt --no-pmc --no-extra --no-cpu-baseline --steps 2 --warmup 1 \
     > $O/kt1_$sc.log 2>&1)
done
echo serial profiles done
