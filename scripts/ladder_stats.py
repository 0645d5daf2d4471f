"""Statistics of the RenderScene progressive ladder against the reference's
result1step/step00000{0..9}.png block means (tests/golden/result1step_blocks.npz).

Renders the 10 launches x 100 spp of CUTracer.cu:378-395 (800x600, scene 1,
the published variant: luminance 30, untinted Fresnel) with the CPU oracle --
bit-identical to the GPU path -- and prints, per step k, the mean and max
|block mean difference| (8-bit units) over the blocks unsaturated in every
reference step.  Used once to set the thresholds of
tests/test_gpu_fullsize.py::test_progressive_ladder_matches_reference_steps.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import oracle
    from montecarlopathtracer_amd.imageio import encode_8bit
    from montecarlopathtracer_amd.scenes import scene_path
    from ladder import ladder_stats
    g = np.load(os.path.join(ROOT, "tests", "golden", "result1step_blocks.npz"))
    s = oracle.Scene(scene_path("scene01"))
    img = np.zeros((600, 800, 3), np.float32)
    for k in range(10):
        p = oracle.RenderParams(width=800, height=600, spp=100, spp_chunk=32, spp_offset=100 * k, prev_count=k,
                                illum=30.0, fresnel_kd=0, threads=int(sys.argv[1]) if len(sys.argv) > 1 else 8)
        img, _ = s.render(p, img)
        m, mx, bias = ladder_stats(encode_8bit(img), g, k)
        print(k, round(m, 4), round(mx, 4), round(bias, 4), flush=True)


if __name__ == "__main__":
    main()
