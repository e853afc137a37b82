"""K03 / K18 / K20 score ops (fp64, deterministic fixed-order reductions).

Each op returns a small device tensor ``res`` (= [ate, se]) so an estimator
can stay on device until its single final read-back. CPU tensors use float64
torch with the same formulas.
"""
from __future__ import annotations

import torch

from .. import _native
from ..parallel import rng
from .panel import dtype_code

NB = 1024  # fixed reduction grid (see csrc/stats.hip)


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _ws(device, *shape):
    return torch.empty(shape, dtype=torch.float64, device=device)


def naive(y: torch.Tensor, w: torch.Tensor, valid: torch.Tensor | None = None):
    """naive_ate (ate_functions.R:3-21) -> (res[2], moments[6])."""
    if not y.is_cuda:
        y64, w64 = y.double(), w.double()
        m = torch.ones_like(y64, dtype=torch.bool) if valid is None else valid.double() != 0
        mom = []
        for g in (0.0, 1.0):
            sel = m & (w64 == g)
            yy = y64[sel]
            mom += [float(sel.sum()), float(yy.sum()), float((yy * yy).sum())]
        mom = torch.tensor(mom, dtype=torch.float64)
        return _naive_finalize(mom), mom
    dev = y.device
    part, mom, res = _ws(dev, NB * 6), _ws(dev, 6), _ws(dev, 2)
    assert y.dtype == w.dtype and (valid is None or valid.dtype == y.dtype)
    _native.call("ate_naive", dtype_code(y), y.data_ptr(), w.data_ptr(),
                 0 if valid is None else valid.data_ptr(), y.numel(), part.data_ptr(),
                 mom.data_ptr(), res.data_ptr(), _stream())
    return res, mom


def _naive_finalize(m):
    n0, s0, q0, n1, s1, q1 = [float(v) for v in m]
    mu0, mu1 = s0 / n0, s1 / n1
    v0 = (q0 - n0 * mu0 * mu0) / (n0 - 1)
    v1 = (q1 - n1 * mu1 * mu1) / (n1 - 1)
    return torch.tensor([mu1 - mu0, (v0 / (n0 - 1) + v1 / (n1 - 1)) ** 0.5], dtype=torch.float64)


def clip_propensity_(p: torch.Tensor, valid: torch.Tensor | None = None):
    """In place: exact 0 -> min positive, exact 1 -> max below one (ate_functions.R:181-182)."""
    if not p.is_cuda:
        m = torch.ones_like(p, dtype=torch.bool) if valid is None else valid.double() != 0
        pv = p[m]
        pos, below = pv[pv > 0], pv[pv < 1]
        if pos.numel():
            p[m & (p == 0)] = pos.min()
        if below.numel():
            p[m & (p == 1)] = below.max()
        return p
    part = _ws(p.device, 2 * NB)
    _native.call("ate_clip_propensity", p.data_ptr(), 0 if valid is None else valid.data_ptr(),
                 p.numel(), part.data_ptr(), _stream())
    return p


def aipw(w, y, p, mu0, mu1, valid=None, compat="reference"):
    """AIPW point + sandwich SE (ate_functions.R:184-199) -> (res[2], moments[6])."""
    sign = 1.0 if compat == "reference" else -1.0
    if not w.is_cuda:
        m = torch.ones_like(w, dtype=torch.bool) if valid is None else valid != 0
        w, y, p, mu0, mu1 = (t.double()[m] for t in (w, y, p, mu0, mu1))
        e1 = w * (y - mu1) / p + sign * (1 - w) * (y - mu0) / (1 - p)
        ok = ~torch.isnan(e1)
        a = w * y / p - mu1 * (w - p) / p - ((1 - w) * y / (1 - p) + mu0 * (w - p) / (1 - p))
        aok = ~torch.isnan(a)
        mom = torch.stack([e1[ok].sum(), ok.sum().double(), (mu1 - mu0).sum(),
                           torch.tensor(float(w.numel()), dtype=torch.float64), a[aok].sum(),
                           (a[aok] ** 2).sum()])
        return _aipw_finalize(mom), mom
    dev = w.device
    part, mom, res = _ws(dev, NB * 6), _ws(dev, 6), _ws(dev, 2)
    _native.call("ate_aipw", w.data_ptr(), y.data_ptr(), p.data_ptr(), mu0.data_ptr(),
                 mu1.data_ptr(), 0 if valid is None else valid.data_ptr(), w.numel(), sign,
                 part.data_ptr(), mom.data_ptr(), res.data_ptr(), _stream())
    return res, mom


def _aipw_finalize(m):
    tau = m[0] / m[1] + m[2] / m[3]
    n = m[3]
    ss = m[5] - 2 * tau * m[4] + n * tau * tau
    return torch.stack([tau, torch.sqrt(torch.clamp(ss, min=0)) / n])


def aipw_terms(w, y, p, mu0, mu1, compat="reference"):
    """Per-row (est1, est2) used by the bootstrap (E10)."""
    sign = 1.0 if compat == "reference" else -1.0
    e1 = w * (y - mu1) / p + sign * (1 - w) * (y - mu0) / (1 - p)
    return e1, mu1 - mu0


def dml_moments(yr, wr, valid=None):
    """[sum wr yr, sum wr^2, sum yr^2 wr^2, sum yr wr^3, sum wr^4, n, sum yr^2]."""
    if not yr.is_cuda:
        m = torch.ones_like(yr, dtype=torch.bool) if valid is None else valid != 0
        y, w = yr.double()[m], wr.double()[m]
        w2 = w * w
        return torch.stack([(w * y).sum(), w2.sum(), (y * y * w2).sum(), (y * w2 * w).sum(),
                            (w2 * w2).sum(), torch.tensor(float(y.numel()), dtype=torch.float64),
                            (y * y).sum()])
    dev = yr.device
    part, mom = _ws(dev, NB * 7), _ws(dev, 7)
    _native.call("ate_dml_moments", yr.data_ptr(), wr.data_ptr(),
                 0 if valid is None else valid.data_ptr(), yr.numel(), part.data_ptr(),
                 mom.data_ptr(), _stream())
    return mom


def dml_moments_exact(yr, wr, dist=None):
    """``dml_moments`` with order-independent sums (ops/exact.py), all-reduced over
    ``dist``: the same bits for any row sharding (bitwise world-size invariance)."""
    from .exact import exact_sum
    y, w = yr.double(), wr.double()
    w2 = w * w
    terms = torch.stack([w * y, w2, y * y * w2, y * w2 * w, w2 * w2, torch.ones_like(y), y * y], 1)
    return exact_sum(terms, dist)


def dml_finalize(mom, mode="plr"):
    """mode 'plr': Neyman-score SE; 'lm': lm(Y_resid ~ 0 + W_resid) SE (ate_functions.R:363)."""
    md = 0 if mode == "plr" else 1
    if not mom.is_cuda:
        n = mom[5]
        theta = mom[0] / mom[1]
        if md == 0:
            j = mom[1] / n
            psi2 = (mom[2] - 2 * theta * mom[3] + theta * theta * mom[4]) / n
            se = torch.sqrt(torch.clamp(psi2, min=0) / (j * j) / n)
        else:
            rss = mom[6] - 2 * theta * mom[0] + theta * theta * mom[1]
            se = torch.sqrt(torch.clamp(rss, min=0) / (n - 1) / mom[1])
        return torch.stack([theta, se])
    res = _ws(mom.device, 2)
    _native.call("ate_dml_finalize", mom.data_ptr(), md, res.data_ptr(), _stream())
    return res


def bootstrap_multinomial(e1, e2, B, seed, b0=0):
    """tau_b for B with-replacement resamples of the FIXED score terms (E10, Q21).
    Draw j of replicate b selects row randint(seed, P_BOOT, b0+b, j, n)."""
    n = e1.numel()
    if not e1.is_cuda:
        import numpy as np
        e1n, e2n = e1.double().numpy(), e2.double().numpy()
        ok = ~np.isnan(e1n)
        e1z = np.where(ok, e1n, 0.0)
        taus = np.empty(B)
        for b in range(B):
            c = rng.bootstrap_counts(n, seed, rng.P_BOOT, b0 + b).astype(np.float64)
            taus[b] = (c @ e1z) / (c @ ok) + (c @ e2n) / n
        return torch.from_numpy(taus)
    taus = _ws(e1.device, B)
    _native.call("ate_boot_multinomial", e1.data_ptr(), e2.data_ptr(), n, seed, b0, B,
                 taus.data_ptr(), _stream())
    return taus


def bootstrap_poisson_partial(e1, e2, B, seed, b0=0, row_offset=0, nb=512):
    """Poisson(1) streaming bootstrap: per-replicate (sum c e1, sum c ok, sum c e2, sum c) over
    this shard's rows -> [B, 4] (all-reduce across ranks, then tau_b = s1/sok + s2/sc)."""
    if not e1.is_cuda:
        raise NotImplementedError("poisson bootstrap is a device op")
    part = _ws(e1.device, nb * ((B + 63) // 64) * 64 * 4)
    _native.call("ate_boot_poisson", e1.data_ptr(), e2.data_ptr(), e1.numel(), seed, b0, B,
                 row_offset, nb, part.data_ptr(), _stream())
    return part.view(nb, -1, 4)[:, :B].sum(0)
