#!/bin/bash
# Round-6 profile set (run on the GPU box via gpurun).  Output under $OUT
# (default gpurun_out/r06):
#   1. the GPU suite + the default bench line with its PMC csv (gpu_check.sh);
#   2. rocprofv3 kernel-trace stats of the C2 frame on one stream (the line's
#      avg_launch_ms agreement) for the reference tree and the SAH tree;
#   3. the phase build (libmcpt_phase.so, -DMCPT_PHASE_TIMING): per-phase wave
#      iterations and lane use of the extend, C2 and C4, one stream.
# Every GPU step has its own time limit; the first failure ends the script.
set -e
R=$PWD
O=${OUT:-gpurun_out/r06}
mkdir -p $O
O=$(cd $O && pwd)
export OUT=$O TMPDIR=/tmp
[ -n "$SKIP_CHECK" ] || bash scripts/gpu_check.sh
for kb in reference sah; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt1_$kb -o run -- \
     python3 $R/bench.py --kd-build $kb --wf-streams 1 --wf-batch 134217728 --no-alt --no-pmc --no-extra \
     --no-cpu-baseline --steps 2 --warmup 1 > $O/kt1_$kb.log 2>&1)
done
echo kernel traces done
for sc in scene01 cornell_bunny70k; do
  MCPT_LIB_PATH=$R/montecarlopathtracer_amd/lib/libmcpt_phase.so timeout -k 10 300 python3 bench.py --scene $sc \
     --no-alt --no-pmc --no-cpu-baseline --no-extra --steps 1 --warmup 0 --wf-streams 1 > $O/phase_$sc.log 2>&1
  grep -h "mcpt lane use\|mcpt phase" $O/phase_$sc.log | tail -2
done
echo phase done
# A/B: the sign-ordered child-box test (MCPT_BOX_SIGN=1, libmcpt_box.so) on C4
LIBS="libmcpt.so libmcpt_box.so" ROUNDS=${AB_ROUNDS:-2} STEPS=10 NOTEST=1 NOPMC=1 OUT=$O/ab_box bash scripts/ab_c4.sh
