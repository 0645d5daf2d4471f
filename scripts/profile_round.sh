#!/bin/bash
# Collect the committed profile set for one round (run on the GPU box via gpurun).
#   $1 = tag (e.g. r01)
# kernel trace + stats, then separate PMC passes (FETCH_SIZE / WRITE_SIZE / SQ
# groups / GRBM), per MI355X_MICROARCH.md "rocprofv3 PMC slots"; then
# scripts/pmc_summary.py folds them into pmc_summary.json.
set -e
TAG=${1:-r01}
R=$PWD
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
# the PMC passes profile the megakernel's path kernel (pmc_summary.py); the
# wavefront (bench's default) gets its kernel trace at the end
B="python3 $R/bench.py --no-cpu-baseline --no-pmc --no-alt ${BENCH_ARGS:---pipeline megakernel}"
timeout -k 10 300 $B --steps 3 --warmup 1 > $OUT/bench.jsonl 2> $OUT/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- $B --steps 2 --warmup 1 > $OUT/kt.log 2>&1
pass() {   # name counters...
  local n=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$n -o run -- $B --steps 1 --warmup 0 > $OUT/$n.log 2>&1
}
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM
pass sq_stall SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS
pass sq_lanes SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_BRANCH SQ_INSTS_VALU_CVT
pass grbm GRBM_GUI_ACTIVE GRBM_COUNT
pass cache TCC_HIT TCC_MISS TCP_TOTAL_CACHE_ACCESSES TCP_TCC_READ_REQ
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_wf -o run -- python3 $R/bench.py --no-cpu-baseline --no-pmc --no-alt --pipeline wavefront --steps 2 --warmup 1 > $OUT/kt_wf.log 2>&1
cd $R
python3 scripts/pmc_summary.py $OUT > $OUT/pmc_summary.json
echo done
