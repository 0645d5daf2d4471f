#!/bin/bash
# Round-3 measurement set (run on the GPU box via gpurun): the default bench
# line with its raw PMC csv kept, a kernel trace of the same workload, the
# N = 2 rehearsals (gloo ranks on one GPU; one process with the device list
# 0,0), each step under its own time limit.
set -e
R=$PWD
O=$R/gpurun_out/r03
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py --keep-pmc $O/pmc > $O/bench.jsonl 2> $O/bench.err
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/bench.py --no-pmc --no-cpu-baseline --no-alt --steps 2 --warmup 1 > $O/kt.log 2>&1
cd $R
MCPT_DIST_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline --no-alt > $O/rehearsal_n2_gloo.jsonl 2> $O/rehearsal_n2_gloo.err
timeout -k 10 300 python3 bench.py --single-process --gpus 2 --devices 0,0 --steps 2 --warmup 1 --no-cpu-baseline --no-alt > $O/rehearsal_n2_single.jsonl 2> $O/rehearsal_n2_single.err
echo done
