#!/bin/bash
# Round-6 fourth set: GPU suite at HEAD (beta/gamma-free accept in the
# queue-order extend), then interleaved A/B against the same build without it
# (libmcpt_bg.so, -DMCPT_WF_NO_BG=0): C2 line + C4 line.
set -e
O=${OUT:-gpurun_out/r06d}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { echo "tests FAILED"; tail -40 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
rm -rf gpurun_out/ab2
LIBS="libmcpt.so libmcpt_bg.so" ROUNDS=3 STEPS=10 NOTEST=1 NOALT=1 ARGS="--no-sah" bash scripts/ab2.sh
mkdir -p $O/ab_bg && cp gpurun_out/ab2/b_*.log $O/ab_bg/
