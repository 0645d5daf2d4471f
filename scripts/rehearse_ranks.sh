#!/bin/bash
# Rehearsal of bench.py's rank path with N ranks sharing this box's GPU(s)
# (gloo for the gather and the timing reductions, as tests/test_gpu_ranks.py at
# N = 2): the full C2 frame, rank 0's PMC passes included, then rank 0's
# gathered image against a one-process render of the same frame.
#   NS="4 8" [SELF=1] bash scripts/rehearse_ranks.sh
# SELF=1: no launcher -- `bench.py --gpus N` starts its own torch.distributed.run
set -e
mkdir -p gpurun_out/rehearse
for n in ${NS:-4 8}; do
  if [ -n "$SELF" ]; then
    MCPT_DIST_BACKEND=gloo timeout -k 10 500 python bench.py --gpus $n --steps 2 --warmup 1 \
      --no-cpu-baseline --dump-image gpurun_out/rehearse/img_n$n.npy > gpurun_out/rehearse/n$n.log 2>&1
  else
    MCPT_DIST_BACKEND=gloo MASTER_ADDR=127.0.0.1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 \
      --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 2 --warmup 1 \
      --no-cpu-baseline --dump-image gpurun_out/rehearse/img_n$n.npy > gpurun_out/rehearse/n$n.log 2>&1
  fi
  grep '^{' gpurun_out/rehearse/n$n.log > gpurun_out/rehearse/n$n.jsonl
done
timeout -k 10 300 python - <<'PY'
import json, os, sys
import numpy as np
import torch
sys.path.insert(0, os.getcwd())
import montecarlopathtracer_amd as M
scene = M.Scene(M.ObjModel(M.scene_path("scene01")))
p = M.RenderParams.for_scene(1, width=1024, height=1024, spp=1024, spp_chunk=32, tile=8)
fb = torch.zeros((p.output_pixels(), 4), dtype=torch.float32, device="cuda:0")
scene.render_device(p, fb.data_ptr(), torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
ref = fb.view(1024, 1024, 4).cpu().numpy()[..., :3]
for n in os.environ.get("NS", "4 8").split():
    ln = json.loads(open(f"gpurun_out/rehearse/n{n}.jsonl").read().splitlines()[-1])
    img = np.load(f"gpurun_out/rehearse/img_n{n}.npy")[..., :3]
    r = ln["roofline"]
    print(json.dumps({"n": int(n), "image_equal": bool(np.array_equal(img, ref)), "value": ln["value"],
                      "ms_per_step": ln["ms_per_step"], "parallelism": ln["config"]["parallelism"],
                      "roofline_frac": r.get("frac"), "binding": r.get("binding"),
                      "rays_per_step": ln["rays_per_step"]}), flush=True)
PY
