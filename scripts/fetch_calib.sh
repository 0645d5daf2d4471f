#!/bin/bash
# FETCH_SIZE calibration (scripts/fetch_calib.hip) and the same counters over
# one C4 frame's kernels (bench.py --pmc-child), one rocprofv3 pass per group.
#   bash scripts/fetch_calib.sh  [OUT=gpurun_out/calib]
set -e
R=$(pwd)
O=$R/${OUT:-gpurun_out/calib}
mkdir -p $O
export TMPDIR=/tmp
rocprofv3 -L > $O/avail.txt 2>&1 || true
P1="FETCH_SIZE"
P2="TCC_EA0_RDREQ TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B"
P3="TCC_EA0_RDREQ_DRAM TCC_EA0_RDREQ_DRAM_32B TCC_BUBBLE"
P4="WRITE_SIZE"
P5="TCC_EA0_WRREQ TCC_EA0_WRREQ_64B TCC_EA0_WR_UNCACHED_32B TCC_EA0_WRREQ_WRITE_DRAM_32B"
i=0
for P in "$P1" "$P2" "$P3" "$P4" "$P5"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $O/calib_p$i -o run -- $R/scripts/_build/fetch_calib > $O/calib_p$i.log 2>&1) || { echo "calib pass $i failed"; tail -5 $O/calib_p$i.log; exit 1; }
done
i=0
for P in "$P1" "$P2" "$P3" "$P4" "$P5"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc $P --output-format csv -d $O/c4_p$i -o run -- python3 $R/bench.py --pmc-child --scene cornell_bunny70k $C4ARGS > $O/c4_p$i.log 2>&1) || { echo "c4 pass $i failed"; tail -5 $O/c4_p$i.log; exit 1; }
done
python3 scripts/fetch_calib_report.py $O
