"""Checkpoint / resume of long runs.

Nuisance predictions per fold and bootstrap replicate ranges are cached as ``.npz``
files keyed by a hash of (stage name, configuration, data fingerprint). Users:

* ``estimators/boosting.py`` (config 5 DML-GBDT, host arrays and HBM panel): the
  held-out E[Y|X], E[W|X] predictions of every finished fold (per rank);
* ``estimators/crossfit.py``: the held-out predictions of every (fold, nuisance) of the
  AIPW cross-fits (config 3, host arrays and HBM panel), and for the causal-forest
  bootstrap (config 4) the forest outputs and each range of bootstrap replicates;
* ``api.replicate``: every finished row of the 14-estimator driver.

Tests kill each of these mid-run and resume to bitwise-identical results
(tests/test_gbdt.py, tests/test_crossfit.py, tests/test_robustness.py). Because all
randomness is counter-based Philox keyed by (seed, purpose, stream, index), a resumed
run reproduces the uninterrupted one bit for bit: completed stages are loaded, the
rest recomputed. Files are written atomically (tmp + rename) and loaded with
``allow_pickle=False``.
"""
from __future__ import annotations

import hashlib
import json
import os
from pathlib import Path

import numpy as np


def fingerprint(*arrays) -> str:
    """Content hash of every byte of every array (blake2b, ~1 GB/s: negligible next to a
    fit). Any edit to the data changes the key, so stale predictions are never reloaded."""
    h = hashlib.blake2b(digest_size=16)
    for a in arrays:
        a = np.ascontiguousarray(np.asarray(a))
        h.update(str(a.shape).encode())
        h.update(str(a.dtype).encode())
        h.update(memoryview(a.reshape(-1).view(np.uint8)))
    return h.hexdigest()


class Checkpoint:
    def __init__(self, directory, config: dict | None = None):
        self.dir = Path(directory)
        self.dir.mkdir(parents=True, exist_ok=True)
        self.config_key = hashlib.sha256(json.dumps(config or {}, sort_keys=True,
                                                    default=str).encode()).hexdigest()[:12]

    def _path(self, stage: str, data_key: str = "") -> Path:
        safe = "".join(c if c.isalnum() or c in "-_." else "_" for c in stage)
        return self.dir / f"{safe}.{self.config_key}.{data_key or 'nodata'}.npz"

    def has(self, stage, data_key=""):
        return self._path(stage, data_key).exists()

    def save(self, stage, data_key="", **arrays):
        p = self._path(stage, data_key)
        tmp = p.with_name(p.name + ".tmp.npz")
        np.savez(tmp, **{k: np.asarray(v) for k, v in arrays.items()})
        os.replace(tmp, p)
        return p

    def load(self, stage, data_key=""):
        with np.load(self._path(stage, data_key), allow_pickle=False) as z:
            return {k: z[k] for k in z.files}

    def cached(self, stage, fn, data_key=""):
        """Return fn()'s dict of arrays, from the cache when this stage already ran."""
        if self.has(stage, data_key):
            return self.load(stage, data_key)
        out = fn()
        self.save(stage, data_key, **out)
        return {k: np.asarray(v) for k, v in out.items()}
