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


def exact_sum(terms: torch.Tensor, dist=None, n_total: int | None = None) -> torch.Tensor:
    """Column sums of ``terms`` [n, m] (fp64; NaN rows excluded by the caller), summed
    over ``dist``'s ranks: identical bits for any row sharding. ``n_total`` bounds the
    number of terms over all ranks (default: dist.n_total, or n)."""
    t = terms.double()
    if t.ndim == 1:
        t = t[:, None]
    n = t.shape[0]
    if n_total is None:
        n_total = dist.n_total if dist is not None else n
    amax = t.abs().amax(0) if n else torch.zeros(t.shape[1], dtype=torch.float64, device=t.device)
    if dist is not None:
        dist.max_(amax)
    sh = _scale_exp(amax, n_total)
    x = torch.ldexp(t, sh[None, :].double()) if hasattr(torch, "ldexp") else t * torch.pow(
        2.0, sh.double())[None, :]
    hi = torch.floor(x)
    lo = torch.round((x - hi) * float(1 << LO_BITS))
    sums = torch.stack([hi.to(torch.int64).sum(0), lo.to(torch.int64).sum(0)])   # [2, m]
    if dist is not None:
        dist.sum_(sums)
    carry = sums[1] >> LO_BITS
    rest = sums[1] - (carry << LO_BITS)
    H = sums[0] + carry
    inv = torch.pow(2.0, -sh.double())
    out = H.double() * inv + rest.double() * (inv * 2.0 ** -LO_BITS)
    bad = ~torch.isfinite(amax)
    return torch.where(bad, torch.full_like(out, float("nan")), out)
