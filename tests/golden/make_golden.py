"""Regenerate the committed golden fixtures (run in the dev container only;
it reads /root/reference, which does not exist on the GPU box).

  <scene>_tinyobj.npz   what the reference's own tinyobjloader v1.1.1
                        (MCRT/QuinEngine/3rdparty/include/tiny_obj_loader.h)
                        reads from each bundled scene, via oracle/_ref/tinyobj_dump
                        built by oracle/ref/Makefile from the reference header.
  result1.png, result1_step000000.png
                        the reference's own renders (CVMCTracer/CVMCTracer/
                        result1.png = 1000 spp, result1step/step000000.png =
                        100 spp), data files copied verbatim.
  oracle_scene01_32x24.npz
                        a small oracle render (regression fixture for the
                        oracle itself; not a reference output).
  mcdocx_fig3_scene2_blinn_phong.png, mcdocx_fig4_scene2_phong.png
                        MC.docx Figures 3 and 4 (word/media/image7.png and
                        image9.png of the .docx zip), byte copies.
  qe_result.png         the reference's own QuinEngine render
                        (MCRT/QuinEngine/result.png, 640x480), byte copy.
  qe_scene01_tinyobj.npz
                        what tinyobjloader reads from QuinEngine's own scene
                        (MCRT/QuinEngine/Res/scene01.obj + its scene01.mtl).
  result1step_blocks.npz
                        50x50-pixel block means (8-bit units) of the reference's
                        progressive ladder result1step/step00000{0..9}.png and
                        the blocks saturated (>= 254) in any step (tests/ladder.py).
"""
import os
import shutil
import struct
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
REF = "/root/reference"


def read_dump(path):
    b = open(path, "rb").read()
    assert b[:4] == b"TOBJ"
    off = 4

    def u32():
        nonlocal off
        v = struct.unpack_from("<I", b, off)[0]
        off += 4
        return v

    def arr(dt, n):
        nonlocal off
        a = np.frombuffer(b, dt, n, off).copy()
        off += 4 * n
        return a

    def s():
        nonlocal off
        n = u32()
        v = b[off:off + n].decode()
        off += n
        return v

    nv = u32(); verts = arr("<f4", 3 * nv).reshape(-1, 3)
    nn = u32(); norms = arr("<f4", 3 * nn).reshape(-1, 3)
    shapes = []
    for _ in range(u32()):
        name = s()
        ni = u32(); idx = arr("<i4", 3 * ni).reshape(-1, 3)
        nf = u32(); mids = arr("<i4", nf)
        shapes.append((name, idx, mids))
    mats = []
    for _ in range(u32()):
        name = s()
        vals = arr("<f4", 12)
        mats.append((name, vals))
    return verts, norms, shapes, mats


def main():
    from montecarlopathtracer_amd.scenes import scene_path
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle", "ref")], check=True)
    tool = os.path.join(ROOT, "oracle", "_ref", "tinyobj_dump")
    for sc in ("scene01", "scene02", "scene03", "qe_scene01"):
        p = scene_path(sc)
        out = f"/tmp/{sc}_tobj.bin"
        subprocess.run([tool, p, os.path.dirname(p) + "/", out], check=True)
        verts, norms, shapes, mats = read_dump(out)
        idx = np.concatenate([x[1] for x in shapes]) if shapes else np.zeros((0, 3), np.int32)
        mids = np.concatenate([x[2] for x in shapes]) if shapes else np.zeros(0, np.int32)
        np.savez_compressed(os.path.join(HERE, f"{sc}_tinyobj.npz"), vertices=verts, normals=norms,
                            indices=idx, material_ids=mids,
                            shape_names=np.array([x[0] for x in shapes]),
                            shape_faces=np.array([len(x[2]) for x in shapes]),
                            mat_names=np.array([m[0] for m in mats]),
                            mat_values=np.stack([m[1] for m in mats]) if mats else np.zeros((0, 12), np.float32))
        print(sc, verts.shape, norms.shape, idx.shape, [x[0] for x in shapes])
    shutil.copy(f"{REF}/CVMCTracer/CVMCTracer/result1.png", os.path.join(HERE, "result1.png"))
    shutil.copy(f"{REF}/CVMCTracer/CVMCTracer/result1step/step000000.png",
                os.path.join(HERE, "result1_step000000.png"))
    # MC.docx figures (a zip member each) and the QuinEngine render, byte copies
    import zipfile
    with zipfile.ZipFile(f"{REF}/MC.docx") as z:
        for member, name in (("word/media/image7.png", "mcdocx_fig3_scene2_blinn_phong.png"),
                             ("word/media/image9.png", "mcdocx_fig4_scene2_phong.png")):
            with open(os.path.join(HERE, name), "wb") as f:
                f.write(z.read(member))
    shutil.copy(f"{REF}/MCRT/QuinEngine/result.png", os.path.join(HERE, "qe_result.png"))
    # the progressive ladder as block means
    from PIL import Image
    sys.path.insert(0, os.path.dirname(HERE))
    from ladder import block_means
    steps = [np.asarray(Image.open(f"{REF}/CVMCTracer/CVMCTracer/result1step/step{k:06d}.png").convert("RGB"))
             for k in range(10)]
    sat = np.zeros(block_means(steps[0]).shape[:2], bool)
    for a in steps:
        sat |= block_means((a >= 254).astype(np.float64)).max(axis=2) > 0
    np.savez_compressed(os.path.join(HERE, "result1step_blocks.npz"),
                        means=np.stack([block_means(a) for a in steps]), saturated=sat)
    import oracle
    s = oracle.Scene(scene_path("scene01"))
    p = oracle.RenderParams(width=32, height=24, spp=4, spp_chunk=2, traversal=oracle.BRUTE, threads=4)
    img, c = s.render(p)
    np.savez_compressed(os.path.join(HERE, "oracle_scene01_32x24.npz"), image=img,
                        counters=np.array([c["rays"], c["paths"], c["shades"]], np.int64))


if __name__ == "__main__":
    main()
