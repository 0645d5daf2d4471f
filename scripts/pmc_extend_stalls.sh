#!/bin/bash
# Where the wavefront extend's wave cycles go (run on the GPU box via gpurun):
# four SQ passes over one C2 render (bench.py --pmc-child), then a per-kernel
# breakdown -- parked on s_waitcnt (WAIT_ANY), issue-stalled (WAIT_INST_ANY),
# issuing (ACTIVE_INST_*), instruction mix per ray.  ARGS adds workload flags.
set -e
R=$PWD
O=$R/gpurun_out/stalls
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
C="python3 $R/bench.py --pmc-child ${ARGS:-}"
pass() {   # name counters...
  local n=$1; shift
  timeout -s KILL 200 rocprofv3 --pmc "$@" --output-format csv -d $O/$n -o run -- $C > $O/$n.log 2>&1
}
pass stall SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS
pass mix SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_THREAD_CYCLES_VALU SQ_BUSY_CYCLES
pass misc SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VMEM SQ_INSTS_SMEM SQ_WAVES GRBM_GUI_ACTIVE
pass lds SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_COUNT
cd $R
python3 scripts/stall_summary.py $O
