"""R-compatible random stream: ``set.seed(s)`` with R's default
generators (Mersenne-Twister, sample.kind "Rejection", R >= 3.6) and ``sample.int``.

Used by the data loader so ``set.seed(1991); sample_n(df, 50000)`` (ate_replication.Rmd:42,
:67) draws the same rows, in the same order, as the reference. Everything else in the
framework uses the counter-based Philox streams (rng.py), which are world-size invariant;
this stream is sequential by definition and host-only.

Algorithms (R's RNG.c / unique.c):
* ``set.seed``: seed <- 50 rounds of ``seed = 69069 * seed + 1`` (mod 2^32), then the 625
  seed words by the same recurrence; word 0 is the MT position (reset to 624), words
  1..624 the MT19937 state.
* ``unif_rand`` = tempered 32-bit MT output * 2^-32, nudged into (0, 1).
* ``R_unif_index(n)``: rejection sampling on ``bits = ceil(log2(n))`` random bits, built
  16 bits at a time from ``floor(unif_rand() * 65536)``.
* ``sample.int(n, k)`` without replacement: the swap-with-last walk over 0..n-1.
"""
from __future__ import annotations

import math

import numpy as np

_I2_32M1 = 2.328306437080797e-10      # 1 / (2^32 - 1)


class RRandom:
    def __init__(self, seed: int):
        s = int(seed) & 0xFFFFFFFF
        for _ in range(50):
            s = (69069 * s + 1) & 0xFFFFFFFF
        words = np.empty(625, dtype=np.uint64)
        for j in range(625):
            s = (69069 * s + 1) & 0xFFFFFFFF
            words[j] = s
        self._bg = np.random.MT19937()
        self._bg.state = {"bit_generator": "MT19937",
                          "state": {"key": words[1:].astype(np.uint32), "pos": 624}}
        self._buf = np.empty(0, dtype=np.uint64)
        self._pos = 0

    def _raw(self) -> int:
        if self._pos >= len(self._buf):
            self._buf = self._bg.random_raw(4096)
            self._pos = 0
        v = int(self._buf[self._pos])
        self._pos += 1
        return v

    def unif_rand(self) -> float:
        x = self._raw() * 2.3283064365386963e-10
        if x <= 0.0:
            return 0.5 * _I2_32M1
        if 1.0 - x <= 0.0:
            return 1.0 - 0.5 * _I2_32M1
        return x

    def runif(self, n: int) -> np.ndarray:
        return np.array([self.unif_rand() for _ in range(n)])

    def _rbits(self, bits: int) -> int:
        v = 0
        for _ in range(0, bits + 1, 16):
            v = 65536 * v + int(math.floor(self.unif_rand() * 65536))
        return v & ((1 << bits) - 1)

    def unif_index(self, n: int) -> int:
        if n <= 0:
            return 0
        bits = int(math.ceil(math.log2(n)))
        while True:
            dv = self._rbits(bits)
            if n > dv:
                return dv

    def sample_int(self, n: int, size: int | None = None) -> np.ndarray:
        """``sample.int(n, size)`` without replacement; 1-based like R."""
        size = n if size is None else int(size)
        if size > n:
            raise ValueError("cannot take a sample larger than the population")
        x = np.arange(n, dtype=np.int64)
        out = np.empty(size, dtype=np.int64)
        m = n
        for i in range(size):
            j = self.unif_index(m)
            out[i] = x[j] + 1
            m -= 1
            x[j] = x[m]
        return out


def r_sample_rows(n: int, size: int, seed: int) -> np.ndarray:
    """0-based row indices of ``set.seed(seed); dplyr::sample_n(df, size)`` (sample order)."""
    return RRandom(seed).sample_int(n, size) - 1


__all__ = ["RRandom", "r_sample_rows"]
