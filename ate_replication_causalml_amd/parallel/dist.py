"""Data-parallel execution context for the estimators (SURVEY.md §2.6 "DP primary").

Rows are sharded contiguously across ranks (rank r holds global rows
[row_offset, row_offset + n_local)). Estimators called with ``dist=DistContext(...)``
build their HBM panel from the local shard and all-reduce every sufficient
statistic — Gram stacks (C01), IRLS Gram + deviance partials (C02), score moments
(C06), bootstrap replicate estimates (C07) — so all ranks finish with the same
estimate, and the result equals the single-device one up to floating-point
summation order (exactly, for the counter-based RNG parts: CV fold ids and
bootstrap draws are keyed by GLOBAL row index).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from . import rng


def shard_range(n_total: int, rank: int, world: int):
    """Balanced contiguous shard: (row_offset, n_local)."""
    base, rem = divmod(n_total, world)
    off = rank * base + min(rank, rem)
    return off, base + (1 if rank < rem else 0)


@dataclass(eq=False)          # identity hash: usable as a static GraphCache argument
class DistContext:
    comm: object
    row_offset: int
    n_total: int

    @classmethod
    def for_rank(cls, comm, n_total: int):
        off, _ = shard_range(n_total, comm.rank, comm.world_size)
        return cls(comm, off, n_total)

    @property
    def capturable(self):
        """Collectives of this context can be captured in a hipGraph (RCCL, world 1)."""
        return self.world == 1 or bool(getattr(self.comm, "capturable", False))

    @property
    def world(self):
        return self.comm.world_size

    @property
    def rank(self):
        return self.comm.rank

    @property
    def n_local(self):
        return shard_range(self.n_total, self.rank, self.world)[1]

    def local(self, a):
        """This rank's rows of a full (replicated) array."""
        return a[self.row_offset:self.row_offset + self.n_local]

    def sum_(self, t: torch.Tensor) -> torch.Tensor:
        return self.comm.all_reduce_(t) if self.world > 1 else t

    def max_(self, t: torch.Tensor) -> torch.Tensor:
        return self.comm.all_reduce_max_(t) if self.world > 1 else t

    def min_(self, t: torch.Tensor) -> torch.Tensor:
        return self.comm.all_reduce_min_(t) if self.world > 1 else t

    def fold_ids(self, K: int, seed: int, stream: int) -> np.ndarray:
        """Global Philox fold assignment (identical to the single-device one), sliced."""
        return self.local(rng.fold_ids(self.n_total, K, seed, stream))

    def gather_rows(self, t: torch.Tensor) -> torch.Tensor:
        """All-gather variable-length row vectors in rank order -> full vector."""
        if self.world == 1:
            return t
        sizes = [shard_range(self.n_total, r, self.world)[1] for r in range(self.world)]
        m = max(sizes)
        buf = torch.zeros((m,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        buf[:t.shape[0]] = t
        parts = self.comm.all_gather(buf)
        return torch.cat([p[:s] for p, s in zip(parts, sizes)])


def maybe_sum_(dist, t):
    return dist.sum_(t) if dist is not None else t
