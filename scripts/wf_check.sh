#!/bin/bash
# wavefront bring-up: parity tests, then bench both pipelines on scene01 and the C4 mesh
set -e
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu -x > gpurun_out/wf_parity.log 2>&1
for pl in megakernel wavefront; do
  timeout -k 10 300 python bench.py --pipeline $pl --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/wf_bench_$pl.log 2>&1
  timeout -k 10 300 python bench.py --pipeline $pl --scene cornell_bunny70k --spp 64 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/wf_bench_c4_$pl.log 2>&1
done
echo done
