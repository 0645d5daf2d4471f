#!/usr/bin/env python3
"""Probe the C ABI's RCCL gather (mcpt_render_params::gather = RCCL) on this box:
a one-device list (a one-rank communicator) and, in a child process under a
time limit, a list that names device 0 twice -- does RCCL accept it?
usage: python scripts/rccl_probe.py [--child DEVLIST]"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def render(devs, gather):
    import numpy as np
    import montecarlopathtracer_amd as M
    M.Tracer().initialize(devs)
    s = M.Scene(M.ObjModel(M.scene_path("scene01")))
    img, st = s.render(M.RenderParams(width=96, height=64, spp=4, gather=gather))
    return np.ascontiguousarray(img), st


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        devs = [int(x) for x in sys.argv[2].split(",")]
        import numpy as np
        ref, _ = render([0], "peer")
        try:
            img, st = render(devs, "rccl")
            print(json.dumps({"devices": devs, "ok": True, "equal": bool(np.array_equal(img, ref)),
                              "n_dev": st["devices"]}))
        except Exception as e:      # McptError: the RCCL message
            print(json.dumps({"devices": devs, "ok": False, "error": str(e)[:400]}))
        return
    out = {}
    for devs in ("0", "0,0"):
        try:
            r = subprocess.run([sys.executable, __file__, "--child", devs], capture_output=True, text=True, timeout=90)
            lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
            out[devs] = json.loads(lines[-1]) if lines else {"rc": r.returncode, "stderr": r.stderr[-600:]}
        except subprocess.TimeoutExpired:
            out[devs] = {"timeout": 90}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
