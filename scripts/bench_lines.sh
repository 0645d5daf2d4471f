#!/bin/bash
# Bench lines for every config (run on the GPU box via gpurun):
#   C2 wavefront (the default) + megakernel, C4 (70k-tri mesh, 1024 spp = BASELINE configs[3]) both pipelines,
#   C5 (wavefront 4096 spp, one GPU), one rank's share at N = 2 / 4 / 8 (scripts/shard_probe.py).
set -e
O=gpurun_out/lines
mkdir -p $O
B="python bench.py --no-cpu-baseline --no-pmc"
BW="python bench.py --no-cpu-baseline"
timeout -k 10 300 $B --pipeline megakernel --no-alt --steps 3 --warmup 1 > $O/c2_megakernel.jsonl 2> $O/c2_megakernel.err
timeout -k 10 300 $B --pipeline megakernel --no-alt --scene cornell_bunny70k --spp 1024 --steps 2 --warmup 1 > $O/c4_megakernel.jsonl 2> $O/c4_megakernel.err
timeout -k 10 400 $BW --scene cornell_bunny70k --spp 1024 --pipeline wavefront --no-alt --steps 2 --warmup 1 > $O/c4_wavefront.jsonl 2> $O/c4_wavefront.err
timeout -k 10 300 $B --spp 4096 --pipeline wavefront --no-alt --steps 1 --warmup 1 > $O/c5_wavefront.jsonl 2> $O/c5_wavefront.err
timeout -k 10 300 python scripts/shard_probe.py 2 4 8 > $O/shard_probe.txt 2>&1
cat $O/shard_probe.txt
for f in $O/*.jsonl; do echo "$f $(grep -o '"value": [0-9.]*' $f | head -1)"; done
