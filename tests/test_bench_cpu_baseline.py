"""bench.py's cpu_baseline legs on the CPU: the all-cores figure renders whole
frames (every pixel) with the oracle, passes continuing the sample sequence."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_all_cores_whole_frames():
    import bench
    r = bench.cpu_all_cores("scene01", 64, 48, 0.2, 2)
    assert r["cores"] == 2 and r["value"] > 0
    assert "whole-frame pass" in r["sample"]
    # at least one pass: every pixel of the 64 x 48 frame shot one path
    rays = int(r["sample"].split(", ")[1].split(" rays")[0])
    assert rays >= 64 * 48


def test_all_cores_single_thread_crops():
    import bench
    r = bench.cpu_all_cores("scene01", 256, 256, 0.1, 1)
    assert r["cores"] == 1 and "centred crop" in r["sample"]
