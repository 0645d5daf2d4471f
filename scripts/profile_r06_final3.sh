#!/bin/bash
# Round-6 closing records at HEAD: the GPU suite, then scripts/profile_r06_final.sh
# (smoke, the driver's bench command with its PMC csv, kernel traces).
set -e
O=${OUT:-gpurun_out/r06final3}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { tail -30 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
OUT=$O bash scripts/profile_r06_final.sh
