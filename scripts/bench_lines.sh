#!/bin/bash
# Bench lines for every config (run on the GPU box via gpurun):
#   C2 wavefront (the default) + megakernel, C4 (70k-tri mesh, 1024 spp = BASELINE configs[3]) both pipelines,
#   C5 (wavefront 4096 spp, one GPU), and a 2-rank rehearsal of the N > 1 path
#   (both ranks on this box's GPU, gloo gather staged through host memory).
set -e
O=gpurun_out/lines
mkdir -p $O
B="python bench.py --no-cpu-baseline --no-pmc"
# wavefront lines carry the per-kernel measured HBM traffic (two PMC passes each)
BW="python bench.py --no-cpu-baseline"
timeout -k 10 400 $BW --pipeline wavefront --no-alt --steps 3 --warmup 1 > $O/c2_wavefront.jsonl 2> $O/c2_wavefront.err
timeout -k 10 300 $B --pipeline megakernel --no-alt --steps 3 --warmup 1 > $O/c2_megakernel.jsonl 2> $O/c2_megakernel.err
timeout -k 10 300 $B --pipeline megakernel --no-alt --scene cornell_bunny70k --spp 1024 --steps 2 --warmup 1 > $O/c4_megakernel.jsonl 2> $O/c4_megakernel.err
timeout -k 10 400 $BW --scene cornell_bunny70k --spp 1024 --pipeline wavefront --no-alt --steps 2 --warmup 1 > $O/c4_wavefront.jsonl 2> $O/c4_wavefront.err
timeout -k 10 300 $B --spp 4096 --pipeline wavefront --no-alt --steps 1 --warmup 1 > $O/c5_wavefront.jsonl 2> $O/c5_wavefront.err
MCPT_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 2 --warmup 1 > $O/rehearsal_n2_gloo.jsonl 2> $O/rehearsal_n2_gloo.err
cat $O/*.jsonl
