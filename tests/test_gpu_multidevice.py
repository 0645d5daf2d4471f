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


@pytest.mark.parametrize("case", range(len(CASES)))
def test_forced_peer_copy_path(mcpt, devices, case):
    """render_multi's cross-device branch (hipMemcpyPeerAsync into devices[0]'s
    gather buffer, capi.cpp) forced between two replicas on one device
    (mcpt_render_params::force_peer_copy): the single-device image bit for bit,
    with a progressive second call and through render_device after reserve."""
    import torch
    kw = dict(CASES[case])
    qe = kw.pop("mode", None) == "qe"
    model = mcpt.ObjModel(mcpt.scene_path("scene01"))
    mk = (lambda **a: mcpt.RenderParams.for_quinengine(**a)) if qe else (lambda **a: mcpt.RenderParams(**a))
    devices([0])
    single = mcpt.Scene(model)
    ref0, _ = single.render(mk(**kw))
    ref1, _ = single.render(mk(spp_offset=kw["spp"], prev_count=1, **kw), ref0.copy())
    devices([0, 0])
    multi = mcpt.Scene(model)
    img0, st = multi.render(mk(force_peer_copy=True, **kw))
    assert st["devices"] == 2
    assert np.array_equal(img0.view(np.uint32), ref0.view(np.uint32))
    img1, _ = multi.render(mk(spp_offset=kw["spp"], prev_count=1, force_peer_copy=True, **kw), img0.copy())
    assert np.array_equal(img1.view(np.uint32), ref1.view(np.uint32))
    p = mk(force_peer_copy=True, **kw)
    multi.reserve(p)
    fb = torch.zeros((p.width * p.height, 4), dtype=torch.float32, device="cuda")
    multi.render_device(p, fb.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    multi.stats()
    assert np.array_equal(fb.view(p.height, p.width, 4)[..., :3].cpu().numpy(), ref0)


def test_init_without_devices_restores_single_device_scenes(mcpt):
    """mcpt_init(NULL, 0) after a device list: later scenes are single-device
    on the current device again (include/mcpt.h)."""
    from montecarlopathtracer_amd._capi import check, lib
    tr = mcpt.Tracer()
    tr.initialize([0, 0])
    model = mcpt.ObjModel(mcpt.scene_path("scene01"))
    assert mcpt.Scene(model).info()["n_devices"] == 2
    check(lib().mcpt_init(None, 0))
    s = mcpt.Scene(model)
    assert s.info()["n_devices"] == 1 and s.info()["device"] == 0
    tr.initialize([0])


def test_plan_query_reports_the_schedule(mcpt, devices):
    """mcpt_plan_query: the automatic scheduling of a render (the bench line's
    config echoes it) and explicit overrides, without allocating anything."""
    devices([0])
    scene = mcpt.Scene(mcpt.ObjModel(mcpt.scene_path("scene01")))
    c2 = dict(width=1024, height=1024, spp=1024, spp_chunk=32)
    wf = scene.plan(mcpt.RenderParams(pipeline="wavefront", **c2))
    assert (wf["pipeline"], wf["variant"], wf["wf_streams"], wf["wf_batch"]) == (1, 4, 3, 1 << 27)
    assert wf["wf_refill"] == 16 and wf["wf_group_shift"] == 6 and wf["work_paths"] == 1 << 30
    # queue order: 2 queues x (3 x 16 + 4 B) + 16 B of radiance = 120 B per path and stream
    assert 3 * 120 * (1 << 27) <= wf["wf_queue_bytes"] < 3 * 121 * (1 << 27) + (1 << 24)
    assert wf["wf_queue_bytes"] <= wf["workspace_bytes"] < wf["device_free_bytes"]
    assert wf["wf_batch_default"] == wf["wf_batch"]          # nothing shrunk on an empty device
    srt = scene.plan(mcpt.RenderParams(pipeline="wavefront", wf_sort=True, **c2))   # (sorts in LDS: same queues)
    assert srt["wf_queue_bytes"] == wf["wf_queue_bytes"]
    mk = scene.plan(mcpt.RenderParams(**c2))
    assert mk["pipeline"] == 0 and mk["ready_thresh"] == 32 and mk["tail_units"] > 0 and mk["variant"] in (1, 2)
    o = scene.plan(mcpt.RenderParams(pipeline="wavefront", wf_streams=2, wf_refill=8, wf_batch=1 << 26, **c2))
    assert (o["wf_streams"], o["wf_refill"], o["wf_batch"]) == (2, 8, 1 << 26)
    devices([0, 0])
    multi = mcpt.Scene(mcpt.ObjModel(mcpt.scene_path("scene01")))
    m = multi.plan(mcpt.RenderParams(pipeline="wavefront", **c2))
    assert m["devices"] == 2 and m["peer_access"] == 1 and m["work_paths"] == (1 << 30) // 2


def test_wavefront_memory_budget(mcpt):
    """wf_mem_limit: a default batch shrinks until its queues fit (same image),
    an explicit batch that does not fit fails with MCPT_E_NOMEM and a message,
    before anything is launched."""
    scene = mcpt.Scene(mcpt.ObjModel(mcpt.scene_path("scene01")))
    kw = dict(width=96, height=64, spp=64, spp_chunk=8, pipeline="wavefront")
    ref, rs = scene.render(mcpt.RenderParams(**kw))
    big = scene.plan(mcpt.RenderParams(**kw))
    lim = big["wf_queue_bytes"] // 2
    small = scene.plan(mcpt.RenderParams(wf_mem_limit=lim, **kw))
    assert small["wf_batch"] < big["wf_batch"]
    # the caller is told: the batch it would have had with memory unbounded
    assert small["wf_batch_default"] == big["wf_batch"] == big["wf_batch_default"]
    img, st = scene.render(mcpt.RenderParams(wf_mem_limit=lim, **kw))
    assert np.array_equal(img, ref) and st["rays"] == rs["rays"]
    with pytest.raises(mcpt.McptError) as e:
        scene.render(mcpt.RenderParams(wf_mem_limit=1 << 20, wf_batch=1 << 20, **kw))
    assert e.value.code == -5 and "wavefront queues" in str(e.value)
    # a reserved scene keeps its reservation: later default-batch renders are
    # fitted into the reserved queue bytes (no re-allocation, e.g. inside a
    # stream capture), with the same image
    fresh = mcpt.Scene(mcpt.ObjModel(mcpt.scene_path("scene01")))
    fresh.reserve(mcpt.RenderParams(wf_mem_limit=lim, **kw))
    after = fresh.plan(mcpt.RenderParams(**kw))
    assert after["wf_batch"] == small["wf_batch"] and after["wf_queue_bytes"] <= lim
    img2, _ = fresh.render(mcpt.RenderParams(**kw))
    assert np.array_equal(img2, ref)


def test_global_layout_option_matches_oracle(mcpt, oracle_mod):
    """MCPT_LAYOUT_GLOBAL (the child-box pair records in global memory) on
    scene01, which would fit in LDS: both pipelines render the oracle's
    node-box walk bit for bit with equal counters."""
    path = mcpt.scene_path("scene01")
    scene = mcpt.Scene(mcpt.ObjModel(path), layout="global")
    assert scene.info()["node_boxes"] == 1 and scene.info()["lds_bytes"] == 0
    W, H, spp, chunk = 48, 40, 6, 3
    ref, rc = oracle_mod.Scene(path).render(oracle_mod.RenderParams(
        width=W, height=H, spp=spp, spp_chunk=chunk, threads=8, node_boxes=1))
    for pipe in ("megakernel", "wavefront"):
        img, st = scene.render(mcpt.RenderParams(width=W, height=H, spp=spp, spp_chunk=chunk, pipeline=pipe))
        assert np.array_equal(img, ref), pipe
        assert st["variant"] == (3 if pipe == "megakernel" else 5)
        for k in ("rays", "paths", "inner_visits", "leaf_visits", "tri_tests", "shades"):
            assert st[k] == rc[k], (pipe, k, st[k], rc[k])


def test_wavefront_render_captured_in_a_graph(mcpt):
    """mcpt_scene_reserve creates the wavefront's side streams and events, so
    a multi-stream wavefront render can be captured into a HIP graph (torch
    CUDA graph on ROCm) and replayed: the replay writes the direct render's
    image."""
    import torch
    scene = mcpt.Scene(mcpt.ObjModel(mcpt.scene_path("scene01")))
    p = mcpt.RenderParams(width=128, height=96, spp=16, spp_chunk=8, pipeline="wavefront", wf_streams=2,
                          wf_batch=128 * 96 * 4)
    ref, _ = scene.render(p)
    scene.reserve(p)
    fb = torch.zeros((128 * 96, 4), dtype=torch.float32, device="cuda")
    s = torch.cuda.Stream()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s, capture_error_mode="relaxed"):
        scene.render_device(p, fb.data_ptr(), s.cuda_stream)
    for _ in range(2):
        fb.zero_()
        g.replay()
    torch.cuda.synchronize()
    assert np.array_equal(fb.view(96, 128, 4)[..., :3].cpu().numpy(), ref)


@pytest.mark.parametrize("pipeline", ["megakernel", "wavefront"])
def test_rccl_gather_one_device(mcpt, devices, pipeline):
    """mcpt_render_params::gather = RCCL (capi.cpp render_multi: ncclCommInitAll
    over mcpt_init's device list, one grouped ncclGather into devices[0]'s
    gather buffer, the unpermute with the running mean) on a one-device list,
    i.e. a one-rank communicator: the plain render's image bit for bit, for a
    progressive second call too and through render_device after reserve.  A
    list naming one GPU twice is refused by RCCL's communicator set-up
    (scripts/rccl_probe.py); two distinct GPUs need the driver's node."""
    import torch
    devices([0])
    scene = mcpt.Scene(mcpt.ObjModel(mcpt.scene_path("scene01")))
    kw = dict(width=67, height=45, spp=5, spp_chunk=2, pipeline=pipeline)
    ref0, st0 = scene.render(mcpt.RenderParams(**kw))
    ref1, _ = scene.render(mcpt.RenderParams(spp_offset=5, prev_count=1, **kw), ref0.copy())
    img0, st = scene.render(mcpt.RenderParams(gather="rccl", **kw))
    assert np.array_equal(img0.view(np.uint32), ref0.view(np.uint32))
    assert st["rays"] == st0["rays"]
    img1, _ = scene.render(mcpt.RenderParams(gather="rccl", spp_offset=5, prev_count=1, **kw), img0.copy())
    assert np.array_equal(img1.view(np.uint32), ref1.view(np.uint32))
    p = mcpt.RenderParams(gather="rccl", **kw)
    scene.reserve(p)
    fb = torch.zeros((45 * 67, 4), dtype=torch.float32, device="cuda")
    scene.render_device(p, fb.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(fb.view(45, 67, 4)[..., :3].cpu().numpy(), ref0)


def test_pw_tracer_dropin_rccl_gather(mcpt, tmp_path):
    """The C++ drop-in (include/mcpt_pw_tracer.hpp) reaching RCCL: Initialize({0})
    + UseRcclGather(true), then the reference's RenderScene loop -- every launch
    a one-rank ncclGather through the C ABI -- renders the Python mirror's image."""
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "cpp"))
    import build_dropin
    exe = build_dropin.build()
    out = str(tmp_path / "img.bin")
    r = subprocess.run([exe, mcpt.scene_path("scene01"), out, "0", "4", "rccl"], capture_output=True, text=True)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr
    got = np.fromfile(out, np.float32).reshape(30, 40, 3)
    tr = mcpt.Tracer()
    tr.initialize([0])
    tr.create_geometry(mcpt.ObjModel(mcpt.scene_path("scene01")))
    host = np.zeros((30, 40, 3), np.float32)
    tr.render_scene(1, host, num_kernels=3, samples_per_kernel=4)
    assert np.array_equal(got, host)


def test_small_reservation_then_larger_render(mcpt):
    """A scene reserved for a small wavefront render (work below one minimum
    batch) still renders a larger one later: the default batch that does not
    fit the reservation grows the workspace from free memory (capi.cpp
    fit_wavefront; only a capturing stream is held to the reservation)."""
    kw = dict(width=96, height=64, spp=64, spp_chunk=8, pipeline="wavefront")
    ref, rs = mcpt.Scene(mcpt.ObjModel(mcpt.scene_path("scene01"))).render(mcpt.RenderParams(**kw))
    scene = mcpt.Scene(mcpt.ObjModel(mcpt.scene_path("scene01")))
    fresh_plan = scene.plan(mcpt.RenderParams(**kw))
    scene.reserve(mcpt.RenderParams(width=16, height=16, spp=2, spp_chunk=2, pipeline="wavefront"))
    assert scene.plan(mcpt.RenderParams(**kw))["wf_batch"] == fresh_plan["wf_batch"]
    img, st = scene.render(mcpt.RenderParams(**kw))
    assert np.array_equal(img, ref) and st["rays"] == rs["rays"]


def test_capture_past_reservation_refused_and_old_graph_survives_growth(mcpt):
    """capi.cpp grow_ws: a render captured into a graph on a scene
    whose reservation is too small fails with MCPT_E_NOMEM before any launch;
    an uncaptured render that grows the workspace retires the reserved buffers
    instead of freeing them, so a graph captured against the reservation still
    replays the right image afterwards; and the grown queues become the
    reservation (a captured render of the larger params is then accepted)."""
    import torch
    from montecarlopathtracer_amd._capi import McptError
    scene = mcpt.Scene(mcpt.ObjModel(mcpt.scene_path("scene01")))
    small = mcpt.RenderParams(width=32, height=32, spp=4, spp_chunk=2, pipeline="wavefront", wf_streams=1)
    big = mcpt.RenderParams(width=96, height=64, spp=64, spp_chunk=8, pipeline="wavefront", wf_streams=1)
    ref_small, _ = scene.render(small)
    ref_big, _ = mcpt.Scene(mcpt.ObjModel(mcpt.scene_path("scene01"))).render(big)
    scene = mcpt.Scene(mcpt.ObjModel(mcpt.scene_path("scene01")))
    scene.reserve(small)
    s = torch.cuda.Stream()
    fb_s = torch.zeros((32 * 32, 4), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    g_small = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g_small, stream=s, capture_error_mode="relaxed"):
        scene.render_device(small, fb_s.data_ptr(), s.cuda_stream)
    # a captured render of the big params: refused, nothing launched
    fb_b = torch.zeros((96 * 64, 4), dtype=torch.float32, device="cuda")
    g_bad = torch.cuda.CUDAGraph()
    err = None
    with torch.cuda.graph(g_bad, stream=s, capture_error_mode="relaxed"):
        try:
            scene.render_device(big, fb_b.data_ptr(), s.cuda_stream)
        except McptError as e:
            err = e
        fb_b.add_(1.0)   # (the graph is not empty)
    assert err is not None and err.code == -5, err   # MCPT_E_NOMEM
    fb_b.zero_()
    g_bad.replay()       # nothing of the refused render was captured
    torch.cuda.synchronize()
    assert bool((fb_b == 1.0).all())
    # uncaptured big render grows the workspace; the small graph still replays correctly
    img, _ = scene.render(big)
    assert np.array_equal(img, ref_big)
    fb_s.zero_()
    g_small.replay()
    torch.cuda.synchronize()
    assert np.array_equal(fb_s.view(32, 32, 4)[..., :3].cpu().numpy(), ref_small)
    # the grown workspace is the reservation now: a captured big render is accepted
    g_big = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g_big, stream=s, capture_error_mode="relaxed"):
        scene.render_device(big, fb_b.data_ptr(), s.cuda_stream)
    fb_b.zero_()
    g_big.replay()
    torch.cuda.synchronize()
    assert np.array_equal(fb_b.view(64, 96, 4)[..., :3].cpu().numpy(), ref_big)


@pytest.mark.parametrize("n", [1, 2])
def test_unknown_gather_rejected_on_every_path(mcpt, devices, n):
    """mcpt_render_params::gather other than PEER / RCCL is MCPT_E_INVALID on a
    one-device scene too, not only where a multi-device render reads it."""
    import ctypes as C
    from montecarlopathtracer_amd._capi import RenderStats, lib
    devices([0] * n)
    scene = mcpt.Scene(mcpt.ObjModel(mcpt.scene_path("scene01")))
    p = mcpt.RenderParams(width=16, height=16, spp=1).to_c()
    p.gather = 2
    fb = np.zeros((16, 16, 3), np.float32)
    st = RenderStats()
    rc = lib().mcpt_render(scene.handle, C.byref(p), fb.ctypes.data_as(C.POINTER(C.c_float)), C.byref(st))
    assert rc == -1, rc   # MCPT_E_INVALID
    assert b"unknown gather" in lib().mcpt_last_error()


def _distinct_gpus():
    try:
        import torch
        return torch.cuda.device_count()
    except Exception:
        return 0


@pytest.mark.skipif(_distinct_gpus() < 2, reason="needs two distinct GPUs (the RCCL gather across devices)")
@pytest.mark.parametrize("pipeline", ["megakernel", "wavefront"])
def test_rccl_gather_two_devices_equals_peer(mcpt, devices, pipeline):
    """The grouped ncclGather across distinct devices (capi.cpp render_multi:
    rank streams, slot-sized send buffers, done events after ncclGroupEnd)
    lands the same image as the peer-copy gather, bit for bit."""
    devices([0, 1])
    scene = mcpt.Scene(mcpt.ObjModel(mcpt.scene_path("scene01")))
    kw = dict(width=67, height=45, spp=5, spp_chunk=2, pipeline=pipeline)
    peer, sp = scene.render(mcpt.RenderParams(gather="peer", **kw))
    rccl, sr = scene.render(mcpt.RenderParams(gather="rccl", **kw))
    assert np.array_equal(rccl.view(np.uint32), peer.view(np.uint32))
    assert sr["rays"] == sp["rays"] and sr["devices"] == 2
