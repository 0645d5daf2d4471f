#!/bin/bash
# memory-pipeline PMC passes for one workload (run on the GPU box):
#   BENCH_ARGS="--scene cornell_bunny70k --spp 256" bash scripts/mem_pmc.sh tag
set -e
TAG=${1:-mem}
R=$PWD
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
B="python3 $R/bench.py --no-cpu-baseline --no-pmc $BENCH_ARGS"
pass() {   # name counters...
  local n=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$n -o run -- $B --steps 1 --warmup 0 > $OUT/$n.log 2>&1
}
pass ta TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES
pass ta2 TA_DATA_STALLED_BY_TC_CYCLES TA_FLAT_READ_WAVEFRONTS
pass tcp TCP_TCC_READ_REQ_LATENCY TCP_TCC_READ_REQ TCP_PENDING_STALL_CYCLES TCP_TCP_LATENCY
pass tcp2 TCP_TOTAL_CACHE_ACCESSES TCP_TCR_TCP_STALL_CYCLES TCP_READ_TAGCONFLICT_STALL_CYCLES TCP_UTCL1_TRANSLATION_MISS
pass sq SQ_WAVE_CYCLES SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
cd $R
echo done
