"""Block statistics of the progressive ladder test (shared by the GPU test and
scripts/ladder_stats.py).  The reference's result1step/step00000k.png is the
8-bit encode (CV/main.cpp:19-29) of the running mean after k+1 launches of
100 samples (CUTracer.cu:378-395); tests/golden/result1step_blocks.npz holds
its 50x50-pixel block means (8-bit units) and, per block, whether any pixel
of any step is saturated (>= 254)."""
import numpy as np

BLOCK = 50


def block_means(img8: np.ndarray) -> np.ndarray:
    H, W, _ = img8.shape
    return img8.astype(np.float64).reshape(H // BLOCK, BLOCK, W // BLOCK, BLOCK, 3).mean(axis=(1, 3))


def ladder_stats(enc8: np.ndarray, golden, k: int):
    """(mean |d|, max |d|, mean d) of our step-k block means vs the reference's,
    8-bit units, over the blocks unsaturated in every reference step"""
    d = (block_means(enc8) - golden["means"][k])[~golden["saturated"]]
    return float(np.abs(d).mean()), float(np.abs(d).max()), float(d.mean())
