"""Multi-GPU behind the C ABI: mcpt_init's device list.

The reference's Initialize() (CUTracer.cu:220-223) picked one device; here
mcpt_init(devices, n) replicates the scene on every listed device and splits
each unsharded render into n interleaved-tile shards, peer-copied to
devices[0] and unpermuted there.  On a one-GPU box the list [0, 0] (and
[0, 0, 0]) puts two (three) replicas on one device: same code path -- replica
streams, shard renders, device-to-device gather, unpermute with the running
mean -- and the image must be the single-device one bit for bit, with the
counters summed over the replicas.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture
def devices(mcpt):
    """set a device list for this test's scenes, restore [0] afterwards"""
    tr = mcpt.Tracer()
    yield tr.initialize
    tr.initialize([0])


CASES = [
    dict(width=67, height=45, spp=5, spp_chunk=2),                         # ragged tiles and chunks
    dict(width=64, height=48, spp=6, spp_chunk=3, pipeline="wavefront"),
    dict(width=40, height=33, spp=4, mode="qe"),
]


@pytest.mark.parametrize("n", [2, 3])
@pytest.mark.parametrize("case", range(len(CASES)))
def test_replicas_render_the_single_device_image(mcpt, devices, n, case):
    kw = dict(CASES[case])
    qe = kw.pop("mode", None) == "qe"
    model = mcpt.ObjModel(mcpt.scene_path("scene01"))
    mk = (lambda **a: mcpt.RenderParams.for_quinengine(**a)) if qe else (lambda **a: mcpt.RenderParams(**a))
    devices([0])
    single = mcpt.Scene(model)
    assert single.info()["n_devices"] == 1
    ref0, st0 = single.render(mk(**kw))
    ref1, _ = single.render(mk(spp_offset=kw["spp"], prev_count=1, **kw), ref0.copy())
    devices([0] * n)
    multi = mcpt.Scene(model)
    assert multi.info()["n_devices"] == n
    img0, st = multi.render(mk(**kw))
    assert np.array_equal(img0.view(np.uint32), ref0.view(np.uint32))
    assert st["devices"] == n
    for k in ("rays", "paths", "shades", "tri_tests", "inner_visits"):
        assert st[k] == st0[k], (k, st[k], st0[k])
    # progressive second call: the gather applies the running mean (linear / gamma)
    img1, _ = multi.render(mk(spp_offset=kw["spp"], prev_count=1, **kw), img0.copy())
    assert np.array_equal(img1.view(np.uint32), ref1.view(np.uint32))
    # explicitly sharded params bypass the split (the caller shards itself)
    part, _ = multi.render(mk(shard_count=2, shard_index=1, **kw))
    ref_part, _ = single.render(mk(shard_count=2, shard_index=1, **kw))
    assert np.array_equal(part, ref_part)


def test_replicas_render_device_async_and_reserve(mcpt, devices):
    """mcpt_render_device on a torch stream + mcpt_scene_reserve, at C1 size."""
    import torch
    devices([0, 0])
    scene = mcpt.Scene(mcpt.ObjModel(mcpt.scene_path("scene01")))
    p = mcpt.RenderParams(width=512, height=512, spp=16, spp_chunk=32, lean=True)
    scene.reserve(p)
    fb = torch.zeros((512 * 512, 4), dtype=torch.float32, device="cuda")
    stream = torch.cuda.current_stream()
    scene.render_device(p, fb.data_ptr(), stream.cuda_stream)
    torch.cuda.synchronize()
    st = scene.stats()
    assert st["devices"] == 2 and st["renders"] == 1 and st["kernel_ms"] > 0
    devices([0])
    single = mcpt.Scene(mcpt.ObjModel(mcpt.scene_path("scene01")))
    ref, rs = single.render(dataclass_replace(p, lean=False))
    assert np.array_equal(fb.view(512, 512, 4)[..., :3].cpu().numpy(), ref)
    assert st["rays"] == rs["rays"]


def dataclass_replace(p, **kw):
    import dataclasses
    return dataclasses.replace(p, **kw)


def test_pw_tracer_dropin_with_device_list(mcpt, tmp_path):
    """The reference-style PW::Tracer call sequence (include/mcpt_pw_tracer.hpp)
    with Initialize({0, 0}): the same image as the Python mirror on one device."""
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "cpp"))
    import build_dropin
    exe = build_dropin.build()
    out = str(tmp_path / "img.bin")
    r = subprocess.run([exe, mcpt.scene_path("scene01"), out, "0,0"], capture_output=True, text=True)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr
    got = np.fromfile(out, np.float32).reshape(30, 40, 3)
    tr = mcpt.Tracer()
    tr.initialize([0])
    tr.create_geometry(mcpt.ObjModel(mcpt.scene_path("scene01")))
    host = np.zeros((30, 40, 3), np.float32)
    tr.render_scene(1, host, num_kernels=3, samples_per_kernel=4)
    assert np.array_equal(got, host)
