#!/bin/bash
# Collect the committed profile set for one round (run on the GPU box via gpurun).
#   $1 = tag (e.g. r01)
# kernel trace + stats, then separate PMC passes (FETCH_SIZE / WRITE_SIZE / SQ),
# per MI355X_MICROARCH.md "rocprofv3 PMC slots".
set -e
TAG=${1:-r01}
R=$PWD
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
B="python3 $R/bench.py --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- $B --steps 2 --warmup 1 > $OUT/kt.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $B --steps 1 --warmup 0 > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $B --steps 1 --warmup 0 > $OUT/write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM --output-format csv -d $OUT/sq -o run -- $B --steps 1 --warmup 0 > $OUT/sq.log 2>&1
echo done
