"""Order-independent (exact) reductions for bitwise reproducibility across world sizes
(SURVEY.md §4.2 "fixed-order reductions", §7.4.5).

A float sum depends on the order of its terms, so a row-sharded estimate would differ
from the single-device one in the last bits. ``exact_sum`` makes every column sum a
function of the SET of terms: each term is split into two int64 fixed-point limbs at a
power-of-two scale chosen from the (exactly all-reduced) column max, the limbs are summed
as integers (associative, so any kernel order, any sharding and any all-reduce algorithm
give the same integers) and recombined once. Resolution is 2^-93 of the largest possible
column sum, far below fp64 rounding of the result. Device-only (no host sync): usable
inside captured graphs, with the all-reduces captured too.
"""
from __future__ import annotations

import torch

HI_BITS = 61          # |sum of hi limbs| < 2^61
LO_BITS = 32          # lo limb in [0, 2^32]


def _scale_exp(amax: torch.Tensor, n_total: float) -> torch.Tensor:
    """Per column: shift sh with amax * n_total * 2^sh < 2^HI_BITS (int64 tensor)."""
    bound = amax.double() * float(max(n_total, 1))
    _, e = torch.frexp(torch.where(bound > 0, bound, torch.ones_like(bound)))   # bound < 2^e
    return (HI_BITS - e.to(torch.int64)).clamp(-1000, 1000)


def column_amax(terms: torch.Tensor) -> torch.Tensor:
    t = terms.double()
    if t.shape[0] == 0:
        return torch.zeros(t.shape[1], dtype=torch.float64, device=t.device)
    return t.abs().amax(0)


def sum_limbs(terms: torch.Tensor, amax: torch.Tensor, n_total: int) -> torch.Tensor:
    """Local int64 limb sums [2, m] of ``terms`` [n, m] at the scale fixed by the GLOBAL
    column max ``amax`` (all-reduced with max) and term count bound ``n_total``."""
    t = terms.double()
    sh = _scale_exp(amax, n_total)
    x = t * torch.pow(2.0, sh.double())[None, :]
    hi = torch.floor(x)
    lo = torch.round((x - hi) * float(1 << LO_BITS))
    return torch.stack([hi.to(torch.int64).sum(0), lo.to(torch.int64).sum(0)])


def finish_limbs(sums: torch.Tensor, amax: torch.Tensor, n_total: int) -> torch.Tensor:
    """fp64 column sums from (all-reduced) limb sums."""
    sh = _scale_exp(amax, n_total)
    carry = sums[1] >> LO_BITS
    rest = sums[1] - (carry << LO_BITS)
    H = sums[0] + carry
    inv = torch.pow(2.0, -sh.double())
    out = H.double() * inv + rest.double() * (inv * 2.0 ** -LO_BITS)
    return torch.where(~torch.isfinite(amax), torch.full_like(out, float("nan")), out)


def exact_sum(terms: torch.Tensor, dist=None, n_total: int | None = None) -> torch.Tensor:
    """Column sums of ``terms`` [n, m] (fp64; NaN rows excluded by the caller), summed
    over ``dist``'s ranks: identical bits for any row sharding. ``n_total`` bounds the
    number of terms over all ranks (default: dist.n_total, or n)."""
    t = terms.double()
    if t.ndim == 1:
        t = t[:, None]
    if n_total is None:
        n_total = dist.n_total if dist is not None else t.shape[0]
    amax = column_amax(t)
    if dist is not None:
        dist.max_(amax)
    sums = sum_limbs(t, amax, n_total)
    if dist is not None:
        dist.sum_(sums)
    return finish_limbs(sums, amax, n_total)


# ---------------------------------------------------------------- fixed-scale limbs
# The exact Gram (ops/gram.py, csrc/gram.hip gram_limbs) splits every chunk partial v into
# hi = floor(v 2^24), lo = rint((v 2^24 - hi) 2^32): int64 sums of the limbs are exact
# for |sum| < 2^38 and resolve 2^-56.
LIMB_HI, LIMB_LO = 24, 32


def to_limbs(v: torch.Tensor) -> torch.Tensor:
    """[2, *v.shape] int64 limbs of fp64 ``v`` (the device rule, bit for bit)."""
    x = v.double() * float(1 << LIMB_HI)
    h = torch.floor(x)
    lo = torch.round((x - h) * float(1 << LIMB_LO))
    return torch.stack([h.to(torch.int64), lo.to(torch.int64)])


def from_limbs(L: torch.Tensor) -> torch.Tensor:
    """fp64 value of summed limbs [2, ...] (deterministic: a function of the integers)."""
    hi, lo = L[0], L[1]
    carry = lo >> LIMB_LO
    rest = lo - (carry << LIMB_LO)
    H = hi + carry
    return (H.double() + rest.double() * 2.0 ** -LIMB_LO) * 2.0 ** -LIMB_HI
