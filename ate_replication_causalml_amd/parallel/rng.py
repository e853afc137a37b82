"""Counter-based Philox4x32-10 RNG shared by the CPU reference path and the HIP kernels.

The reference relies on R's global Mersenne-Twister stream (``set.seed(1991)``,
``ate_replication.Rmd:42``) for fold ids, bootstrap resamples
(``ate_functions.R:269``) and randomForest bootstraps. A single sequential
stream cannot be split across GPUs deterministically, so every random draw in
this framework is a pure function of ``(seed, purpose, stream, index)``:

    counter = (index_lo, index_hi, purpose, stream), key = (seed_lo, seed_hi)

The identical function is implemented in ``csrc/philox.hpp`` so that a draw
made on the CPU reference path and on any GPU of any world size is
bit-identical.
"""
from __future__ import annotations

import numpy as np

M0 = np.uint64(0xD2511F53)
M1 = np.uint64(0xCD9E8D57)
W0 = np.uint32(0x9E3779B9)
W1 = np.uint32(0xBB67AE85)
_MASK32 = np.uint64(0xFFFFFFFF)

# purposes (counter word 2). Keep in sync with csrc/philox.hpp.
P_FOLD = 1          # cross-fit / CV fold assignment
P_BOOT = 2          # AIPW bootstrap replicate resampling (E10)
P_RF_BOOT = 3       # random forest bootstrap sample per tree
P_RF_MTRY = 4       # per-node feature subsampling
P_DGP = 5           # synthetic data generation
P_SUBSAMPLE = 6     # grf half-sampling / honesty split
P_GBDT = 7          # GBDT row/feature subsampling
P_SAMPLE_ROWS = 8   # sample_n row selection in the data pipeline


def philox4x32(c0, c1, c2, c3, k0, k1, rounds: int = 10):
    """Vectorised Philox4x32 over uint32 numpy arrays (broadcasting)."""
    c0 = np.asarray(c0, dtype=np.uint32).astype(np.uint64)
    c1 = np.asarray(c1, dtype=np.uint32).astype(np.uint64)
    c2 = np.asarray(c2, dtype=np.uint32).astype(np.uint64)
    c3 = np.asarray(c3, dtype=np.uint32).astype(np.uint64)
    c0, c1, c2, c3 = np.broadcast_arrays(c0, c1, c2, c3)
    k0 = np.uint64(np.uint32(k0))
    k1 = np.uint64(np.uint32(k1))
    for _ in range(rounds):
        p0 = M0 * c0
        p1 = M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & _MASK32
        hi1, lo1 = p1 >> np.uint64(32), p1 & _MASK32
        n0 = hi1 ^ c1 ^ k0
        n2 = hi0 ^ c3 ^ k1
        c0, c1, c2, c3 = n0, lo1, n2, lo0
        k0 = (k0 + np.uint64(W0)) & _MASK32
        k1 = (k1 + np.uint64(W1)) & _MASK32
    return (c0.astype(np.uint32), c1.astype(np.uint32),
            c2.astype(np.uint32), c3.astype(np.uint32))


def _split_seed(seed: int):
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    return seed & 0xFFFFFFFF, seed >> 32


def random_u32(seed: int, purpose: int, stream, index):
    """Four uint32 words per (stream, index). Returns array shape (..., 4)."""
    index = np.asarray(index, dtype=np.uint64)
    k0, k1 = _split_seed(seed)
    lo = (index & _MASK32).astype(np.uint32)
    hi = (index >> np.uint64(32)).astype(np.uint32)
    out = philox4x32(lo, hi, np.uint32(purpose), np.asarray(stream, dtype=np.uint32), k0, k1)
    return np.stack(out, axis=-1)


def uniform(seed: int, purpose: int, stream, index, word: int = 0):
    """U[0,1) float with 24 random bits (exactly representable in fp32)."""
    u = random_u32(seed, purpose, stream, index)[..., word]
    return (u >> np.uint32(8)).astype(np.float64) * (1.0 / 16777216.0)


def randint(seed: int, purpose: int, stream, index, n: int, word: int = 0):
    """Uniform integer in [0, n) via 32x32->64 multiply-shift (same on device)."""
    u = random_u32(seed, purpose, stream, index)[..., word].astype(np.uint64)
    return ((u * np.uint64(n)) >> np.uint64(32)).astype(np.int64)


def normal_pair(seed: int, purpose: int, stream, index):
    """Two N(0,1) draws per index via Box-Muller on words (0,1) and (2,3)."""
    w = random_u32(seed, purpose, stream, index).astype(np.float64)
    u1 = (np.floor(w[..., 0] / 256.0) + 1.0) * (1.0 / 16777217.0)  # (0,1]
    u2 = np.floor(w[..., 1] / 256.0) * (1.0 / 16777216.0)
    r = np.sqrt(-2.0 * np.log(u1))
    return r * np.cos(2 * np.pi * u2), r * np.sin(2 * np.pi * u2)


def fold_ids(n: int, k: int, seed: int, stream: int = 0) -> np.ndarray:
    """Balanced random fold assignment (the analogue of glmnet's
    ``sample(rep(seq(nfolds), length = N))``): a Philox-keyed random
    permutation of ``arange(n) % k``. Deterministic and world-size independent."""
    keys = random_u32(seed, P_FOLD, stream, np.arange(n, dtype=np.uint64))
    key = (keys[..., 0].astype(np.uint64) << np.uint64(32)) | keys[..., 1].astype(np.uint64)
    order = np.argsort(key, kind="stable")
    folds = np.empty(n, dtype=np.int64)
    folds[order] = np.arange(n) % k
    return folds


def bootstrap_counts(n: int, seed: int, purpose: int, stream: int) -> np.ndarray:
    """Multinomial(n; 1/n) counts of a with-replacement resample of size n.
    Draw j picks row randint(seed, purpose, stream, j, n) (K10)."""
    idx = randint(seed, purpose, stream, np.arange(n, dtype=np.uint64), n)
    return np.bincount(idx, minlength=n)
