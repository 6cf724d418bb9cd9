"""Portable counter-based RNG — TEST INFRASTRUCTURE (oracle side).

This is the numpy restatement of the device generator in
``<pkg>/csrc/rng.h``.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import anything under ``oracle/``.

Why it exists: the reference draws its dropout masks and the VAE noise from
the torch CPU generator in module order (causal_anomaly_detection.py:330 for
``randn_like``; nn.Dropout inside detector_net cad:170,173, causal_scorer
cad:438 and direct_classifier cad:528,531).  A GPU build cannot replay that
stream, so both sides draw from this keyed hash instead: every random value is
a pure function of (seed, stream, step, row, col).  Rows are GLOBAL frame/clip
indices, so a data-parallel run draws the same values as a single process.

Contract (bit-exact between numpy and HIP):
    mix(z)   = splitmix64 finaliser
    h0       = mix(seed + GOLDEN * (stream + 1))
    h1       = mix(h0 ^ step)
    h(r, c)  = mix(h1 ^ ((r << 32) | c))
    u24      = h >> 40                      (uniform integer in [0, 2^24))
    keep     = u24 >= floor(p * 2^24)      (dropout; scale 1/(1-p) on keep)
    eps      = sqrt(-2 ln((u24(2i)+1)/2^24)) * cos(2 pi u24(2i+1)/2^24)   (f64 → f32)
    pixel u8 = h >> 56
"""
from __future__ import annotations

import numpy as np

GOLDEN = np.uint64(0x9E3779B97F4A7C15)
M1 = np.uint64(0xBF58476D1CE4E5B9)
M2 = np.uint64(0x94D049BB133111EB)

# stream ids (must match csrc/rng.h)
S_INPUT = 1
S_DET_DROP1 = 2
S_DET_DROP2 = 3
S_EPS = 4
S_SCORER_DROP = 5
S_DIRECT_DROP1 = 6
S_DIRECT_DROP2 = 7
S_MC_DROP1 = 8
S_MC_DROP2 = 9
S_A2_DROP_FC = 10
S_A2_DROP_GRAPH = 11
S_A2_PSEUDO = 12
S_BBOX_DROP = 13


def _mix(z):
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * M1
        z = (z ^ (z >> np.uint64(27))) * M2
    return z ^ (z >> np.uint64(31))


def _h1(seed: int, stream: int, step: int) -> np.uint64:
    with np.errstate(over="ignore"):
        z = np.uint64(seed % (1 << 64)) + GOLDEN * np.uint64(stream + 1)
    h0 = _mix(z)
    return _mix(h0 ^ np.uint64(step))


def hash_grid(seed: int, stream: int, step: int, rows, cols) -> np.ndarray:
    """uint64 hashes for every (row, col) of the outer product rows × cols."""
    r = np.asarray(rows, dtype=np.uint64).reshape(-1, 1)
    c = np.asarray(cols, dtype=np.uint64).reshape(1, -1)
    h1 = _h1(seed, stream, step)
    return _mix(h1 ^ ((r << np.uint64(32)) | c))


def u24(seed, stream, step, rows, cols) -> np.ndarray:
    return (hash_grid(seed, stream, step, rows, cols) >> np.uint64(40)).astype(np.int64)


def dropout_keep(seed: int, stream: int, step: int, row0: int, nrows: int, ncols: int, p: float) -> np.ndarray:
    """bool keep-mask (nrows, ncols) for global rows row0..row0+nrows-1."""
    thr = int(np.floor(p * 16777216.0))
    return u24(seed, stream, step, np.arange(row0, row0 + nrows), np.arange(ncols)) >= thr


def dropout_scale(p: float) -> np.float32:
    return np.float32(1.0) / np.float32(1.0 - p)


def normal_eps(seed: int, stream: int, step: int, row0: int, nrows: int, nelem: int) -> np.ndarray:
    """float32 N(0,1) draws (nrows, nelem) by Box-Muller over pairs of u24."""
    u = u24(seed, stream, step, np.arange(row0, row0 + nrows), np.arange(2 * nelem))
    u1 = (u[:, 0::2].astype(np.float64) + 1.0) / 16777216.0
    u2 = u[:, 1::2].astype(np.float64) / 16777216.0
    return (np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * np.pi * u2)).astype(np.float32)


def pixels_u8(seed: int, step: int, row0: int, nrows: int, npix: int) -> np.ndarray:
    """uint8 synthetic pixels (nrows, npix); row = global frame index."""
    h = hash_grid(seed, S_INPUT, step, np.arange(row0, row0 + nrows), np.arange(npix))
    return (h >> np.uint64(56)).astype(np.uint8)


def uniform01(seed: int, stream: int, step: int, row0: int, nrows: int, ncols: int) -> np.ndarray:
    """float32 uniform [0,1) with 24-bit resolution (used for a2 pseudo-labels)."""
    u = u24(seed, stream, step, np.arange(row0, row0 + nrows), np.arange(ncols))
    return (u.astype(np.float64) / 16777216.0).astype(np.float32)
