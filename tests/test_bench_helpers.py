"""bench.py's host-side accounting (no GPU): SURVEY 8(d)'s bytes model and the
rocprofv3 csv readers behind roofline.traffic / roofline.kernels, on small
synthetic counter files in rocprofv3's csv layout."""
import csv
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

HEADER = ["Correlation_Id", "Dispatch_Id", "Agent_Id", "Queue_Id", "Process_Id", "Thread_Id", "Grid_Size",
          "Kernel_Id", "Kernel_Name", "Workgroup_Size", "LDS_Block_Size", "Scratch_Size", "VGPR_Count",
          "Accum_VGPR_Count", "SGPR_Count", "Counter_Name", "Counter_Value", "Start_Timestamp", "End_Timestamp"]


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _write(d, rows):
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "run_counter_collection.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(HEADER)
        for disp, name, cn, val, t0, t1 in rows:
            w.writerow([disp, disp, "Agent 2", 1, 1, 1, 1024, 7, name, 256, 0, 0, 64, 0, 16, cn, val, t0, t1])


def test_algorithmic_bytes_is_survey_formula():
    b = _bench()
    st = {"inner_visits": 10, "leaf_visits": 2, "leaf_refs": 3, "tri_tests": 3, "shades": 1}
    ab = b.algorithmic_bytes(st, pixels=4)
    assert ab["survey"] == 32 * 12 + 4 * 3 + 48 * 3 + 96 * 1 + 16 * 4
    assert ab["own"] == 8 * 12 + 4 * 3 + 48 * 3 + 96 * 1 + 16 * 4


def test_wavefront_kernel_reader_sums_dispatches(tmp_path):
    b = _bench()
    ext = "void mcpt::(anonymous namespace)::wf_extend<true, 4, 1024>(mcpt::KernelParams, mcpt::WfParams)"
    shd = "void mcpt::(anonymous namespace)::wf_shade_slots<1024>(mcpt::KernelParams, mcpt::WfParams)"
    other = "void at::native::vectorized_elementwise_kernel<4>(int)"
    # counters summed over XCD rows of one dispatch, then over dispatches; time per dispatch once
    _write(str(tmp_path / "p"), [
        (1, ext, "FETCH_SIZE", 100.0, 1000, 3000), (1, ext, "FETCH_SIZE", 50.0, 1000, 3000),
        (2, ext, "FETCH_SIZE", 10.0, 5000, 6000),
        (3, shd, "FETCH_SIZE", 7.0, 7000, 7500),
        (4, other, "FETCH_SIZE", 1e9, 0, 10),
    ])
    r = b.read_wf_kernels(str(tmp_path / "p"))
    assert set(r) == {"extend", "shade"}
    assert r["extend"]["FETCH_SIZE"] == 160.0 and r["extend"]["ns"] == 3000 and r["extend"]["dispatches"] == 2
    assert r["shade"]["FETCH_SIZE"] == 7.0 and r["shade"]["ns"] == 500


def test_path_kernel_reader_picks_the_lean_kernel(tmp_path):
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    from pmc_summary import read_counters
    lean = "void mcpt::(anonymous namespace)::path_kernel<true, 4, 1024, false, false, false>(mcpt::KernelParams)"
    counting = "void mcpt::(anonymous namespace)::path_kernel<true, 4, 1024, false, false, true>(mcpt::KernelParams)"
    _write(str(tmp_path / "q"), [
        (1, counting, "WRITE_SIZE", 999.0, 0, 1),
        (2, lean, "WRITE_SIZE", 4.0, 0, 1), (2, lean, "WRITE_SIZE", 6.0, 0, 1),
        (3, lean, "WRITE_SIZE", 20.0, 0, 1),
    ])
    # per-launch average over the lean kernel's dispatches: (10 + 20) / 2
    assert read_counters(str(tmp_path / "q")) == {"WRITE_SIZE": 15.0}


def test_lds_block_and_binding_roof():
    b = _bench()
    cus = 256
    # 1e6 kernel cycles (GRBM summed over 8 XCDs), LDS array busy 0.4 of every CU's cycles
    pmc = {"SQ_LDS_IDX_ACTIVE": 0.4 * cus * 1e6, "GRBM_GUI_ACTIVE": 8e6, "SQ_INSTS_LDS": 1e6,
           "SQ_LDS_BANK_CONFLICT": 2.5e6, "ns": 1e6}
    per = {"inner_visits": 1e6, "leaf_refs": 2e5, "tri_tests": 3e5}
    lb = b.lds_block(pmc, cus, per)
    assert lb["array_busy_frac"] == 0.4
    assert lb["traffic"] == round((16e6 + 4 * 2e5 + 48 * 3e5) / 1e9, 3)
    assert lb["achieved"] == round((16e6 + 8e5 + 1.44e7) / 1e6, 1)      # bytes / ns = GB/s
    assert lb["conflict_cycles_per_lds_instr"] == 2.5
    bd = b.binding_of({"frac": 0.08, "lds": lb, "valu": {"issue_frac": 0.55}})
    assert bd["binding"] == "valu_issue" and bd["binding_frac"] == 0.55
    assert set(bd["fracs"]) == {"hbm", "lds_array", "valu_issue"}
    assert b.binding_of({"frac": 0.9, "lds": lb})["binding"] == "hbm"
    assert b.lds_block({}, cus, per) == {}


def test_ray_stream_bytes():
    """bench.ray_stream_bytes: 32 B per secondary ray; bounce 0 reads 16 B per
    path except on the LDS wavefront (variant 4), whose packet extend computes
    its primary rays."""
    import bench
    assert bench.ray_stream_bytes(10, 4, 5) == 16 * 4 + 32 * 6
    assert bench.ray_stream_bytes(10, 4, 4) == 32 * 6


def test_ray_stream_bytes_qe():
    """in QuinEngine mode there is no implicit bounce 0 -- the
    extend reads both streams of every primary ray; hit ids are 4 B (the
    material sort, which sorts inside the shade, included)."""
    bench = _bench()
    for v in (4, 5):
        assert bench.ray_stream_bytes(10, 4, v, qe=True) == 32 * 10
    assert bench.hit_write_bytes(10) == 40


def _run_bench(args, env_extra, timeout=120):
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MCPT_DIST_BACKEND")}
    env.update(env_extra)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          timeout=timeout, env=env, cwd=ROOT)


def test_bench_refuses_more_gpus_than_visible():
    """`bench.py --gpus N` without a launcher starts N ranks
    itself, and exits non-zero (no JSON line) when fewer than N GPUs are
    visible -- here none -- instead of measuring one GPU and calling it N."""
    import torch
    if torch.cuda.device_count() >= 2:
        import pytest
        pytest.skip("enough GPUs: the launcher would run")
    r = _run_bench(["--gpus", "2", "--steps", "1", "--warmup", "0"], {})
    assert r.returncode != 0
    assert "GPU(s) visible" in r.stderr, r.stderr[-2000:]
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_bench_refuses_world_size_mismatch():
    """A launcher that started a different number of ranks than --gpus: exit
    non-zero before any GPU call (no line whose n_gpus differs from --gpus)."""
    r = _run_bench(["--gpus", "2", "--steps", "1"], {"WORLD_SIZE": "3", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=3" in r.stderr, r.stderr[-2000:]
    r = _run_bench(["--gpus", "1", "--steps", "1"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr, r.stderr[-2000:]


def test_pmc_child_replays_the_line_s_scene_options():
    """The PMC passes profile the same render as the line: the child's argument
    list carries the KD split rule and the material sort (bench._workload_args)."""
    import argparse
    bench = _bench()
    a = argparse.Namespace(scene="scene01", width=64, height=48, spp=4, spp_chunk=2, pipeline="wavefront",
                           wf_batch=0, wf_streams=0, layout="auto", set=[], counting=False, wf_sort=True,
                           kd_build="sah")
    w = bench._workload_args(a, (2, 1))
    assert w[w.index("--kd-build") + 1] == "sah" and "--wf-sort" in w
    assert w[w.index("--pmc-shard") + 1] == "2,1"
