"""Price VERDICT r05 item 2 on the CPU oracle (no GPU): for the secondary rays of
a C2 / C4 sample, the ordered walk's first-descent inner steps and how many of
them a replay of the previous hit leaf's ancestor chain would serve (see
scripts/price_descent.c).  Diagnostic only.

  python scripts/price_descent.py [scene01|cornell_bunny70k] [crop] [spp]
"""
import ctypes as C
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
SO = "/tmp/mcpt_price_descent.so"


def build():
    subprocess.run(["gcc", "-O2", "-std=gnu99", "-ffp-contract=off", "-shared", "-fPIC", "-o", SO,
                    os.path.join(ROOT, "scripts", "price_descent.c"), os.path.join(ROOT, "oracle", "obj_reader.c"),
                    os.path.join(ROOT, "oracle", "kdtree_ref.c"), "-I", os.path.join(ROOT, "oracle"), "-lm",
                    "-pthread"], check=True)


def main():
    scene = sys.argv[1] if len(sys.argv) > 1 else "scene01"
    crop = int(sys.argv[2]) if len(sys.argv) > 2 else 128
    spp = int(sys.argv[3]) if len(sys.argv) > 3 else 16
    build()
    import oracle
    oracle.LIB_PATH = SO
    L = oracle.lib()
    L.diag_init.argtypes = [C.c_void_p]
    L.diag_read.argtypes = [C.POINTER(C.c_double)]
    from montecarlopathtracer_amd.scenes import scene_path
    s = oracle.Scene(scene_path(scene))
    L.diag_init(s._h)
    # crop > 0: a centred crop of the 1024^2 frame; crop < 0: the whole frame at
    # |crop| x |crop| pixels (the same view, every region sampled)
    W = H = 1024 if crop > 0 else -crop
    crop = crop if crop > 0 else W
    x0, y0 = (W - crop) // 2, (H - crop) // 2
    boxes = 1 if scene != "scene01" else 0
    p = oracle.RenderParams(width=W, height=H, spp=spp, spp_chunk=32, traversal=oracle.KD_ORDERED, threads=1,
                            region=(x0, y0, x0 + crop, y0 + crop), node_boxes=boxes)
    _, c = s.render(p)
    out = (C.c_double * 200)()
    L.diag_read(out)
    rays, first, served, s4, s8, same = (out[i] for i in range(6))
    hist = np.array([out[6 + i] for i in range(97)])
    print(f"{scene} crop {crop} spp {spp} node_boxes {boxes}: rays {c['rays']} secondary {int(rays)}")
    print(f"  inner visits/ray (all rays) {c['inner_visits'] / c['rays']:.2f}  leaf {c['leaf_visits'] / c['rays']:.2f}"
          f"  tri tests {c['tri_tests'] / c['rays']:.2f}")
    print(f"  secondary: first-descent inner steps {first / rays:.2f}, on the prev-leaf chain {served / rays:.2f}"
          f" ({served / max(first, 1):.1%}); exact chain {same / rays:.1%}")
    print(f"  dependent round trips saved per secondary ray: groups of 4 {s4 / rays:.2f}, groups of 8 {s8 / rays:.2f}")
    cum = np.cumsum(hist) / rays
    print("  served-steps CDF:", " ".join(f"{i}:{cum[i]:.2f}" for i in range(0, 33, 4)))


if __name__ == "__main__":
    main()
