"""K05/K06/K07 ops: rank-revealing normal-equation solve, GEMV predictors, logistic IRLS.

GPU kernels: ``csrc/linalg.hip``. CPU: float64 numpy/torch with identical
semantics (used by CPU tests and as the kernels' numerics reference).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from .. import _native
from .devconst import const
from .gram import gram
from .panel import DevicePanel, dtype_code

LM_TOL = 1e-7


def logistic(x: torch.Tensor) -> torch.Tensor:
    """1 / (1 + exp(-x)) with a result that depends on each element alone. On the CPU,
    torch.sigmoid's vectorised body and its scalar tail round differently, so the same row
    got a different last bit depending on where a rank's shard ended (world 8, found by
    tests/test_world8.py); exp and the division are exact per element in every lane. GPU
    tensors keep torch.sigmoid (no tail path: one formula per element)."""
    if x.is_cuda:
        return torch.sigmoid(x)
    return torch.reciprocal(1.0 + torch.exp(-x))


def _stream():
    return torch.cuda.current_stream().cuda_stream


@dataclass
class SolveResult:
    beta: torch.Tensor       # (k,) fp64, NaN = aliased
    invdiag: torch.Tensor    # (k,) diag((X'X)^-1) restricted to non-aliased
    aux: torch.Tensor        # (4,) rank, rss (= y'y - b'X'y), y'y, 0


class SolveWorkspace:
    def __init__(self, k, device):
        self.work = torch.empty(2 * k * k, dtype=torch.float64, device=device)
        self.beta = torch.zeros(k, dtype=torch.float64, device=device)
        self.invdiag = torch.empty(k, dtype=torch.float64, device=device)
        self.aux = torch.empty(4, dtype=torch.float64, device=device)


def chol_solve(G: torch.Tensor, cols, rcol: int = -1, rhs: torch.Tensor | None = None,
               tol: float = LM_TOL, done: torch.Tensor | None = None,
               ws: SolveWorkspace | None = None) -> SolveResult:
    """Solve G[cols,cols] b = G[cols,rcol] (or rhs) with column-order aliasing (lm rule)."""
    cols_t = cols if isinstance(cols, torch.Tensor) else const(cols, torch.int32, G.device)
    k = cols_t.numel()
    if not G.is_cuda:
        return _chol_solve_cpu(G, cols_t.cpu().numpy(), rcol, rhs, tol)
    ws = ws or SolveWorkspace(k, G.device)
    _native.call("ate_chol_solve", G.data_ptr(), G.shape[-1], cols_t.data_ptr(), k, rcol,
                 0 if rhs is None else rhs.data_ptr(), tol, ws.work.data_ptr(), ws.beta.data_ptr(),
                 ws.invdiag.data_ptr(), ws.aux.data_ptr(),
                 0 if done is None else done.data_ptr(), _stream())
    return SolveResult(ws.beta, ws.invdiag, ws.aux)


def spd_solve(K: torch.Tensor, r: torch.Tensor) -> torch.Tensor:
    """x[a] = K[a]^-1 r[a] for a batch [A, k, k] of small SPD systems (unpivoted Cholesky;
    NaN for a system without a positive pivot). GPU: csrc/linalg.hip spd_solve_kernel, a
    kernel of ours so the solve can sit inside a hipGraph (torch.linalg.cholesky_ex cannot
    be captured on ROCm); CPU: torch.linalg."""
    if not K.is_cuda:
        L, info = torch.linalg.cholesky_ex(K)
        x = torch.cholesky_solve(r[:, :, None], L)[:, :, 0]
        return torch.where((info > 0)[:, None], torch.full_like(x, float("nan")), x)
    A, k = K.shape[0], K.shape[-1]
    Kc = K.contiguous().double()
    rc = r.contiguous().double()
    work = torch.empty(A * k * k, dtype=torch.float64, device=K.device)
    x = torch.empty(A, k, dtype=torch.float64, device=K.device)
    _native.call("ate_spd_solve_batched", Kc.data_ptr(), rc.data_ptr(), A, k, work.data_ptr(),
                 x.data_ptr(), _stream())
    return x


def chol_solve_active(G: torch.Tensor, cols: torch.Tensor, kact: torch.Tensor, rcol: int,
                      tol: float = LM_TOL, ws: SolveWorkspace | None = None) -> SolveResult:
    """chol_solve over the first ``kact`` (device int32 scalar) entries of the device column
    list ``cols`` (fixed length): a data-dependent design size without a host sync. Entries
    of beta / invdiag past kact are unspecified; aux counts the active columns only."""
    k = cols.numel()
    if not G.is_cuda:
        ka = int(kact)
        r = _chol_solve_cpu(G, cols[:ka].cpu().numpy(), rcol, None, tol)
        pad = torch.full((k - ka,), float("nan"), dtype=torch.float64)
        return SolveResult(torch.cat([r.beta.cpu(), pad]), torch.cat([r.invdiag.cpu(), pad]), r.aux)
    ws = ws or SolveWorkspace(k, G.device)
    _native.call("ate_chol_solve_k", G.data_ptr(), G.shape[-1], cols.data_ptr(), k, kact.data_ptr(),
                 rcol, tol, ws.work.data_ptr(), ws.beta.data_ptr(), ws.invdiag.data_ptr(),
                 ws.aux.data_ptr(), _stream())
    return SolveResult(ws.beta, ws.invdiag, ws.aux)


def _chol_solve_cpu(G, cols, rcol, rhs, tol):
    Gn = G.detach().cpu().double().numpy()
    A = Gn[np.ix_(cols, cols)].copy()
    b = (Gn[cols, rcol] if rhs is None else rhs.cpu().double().numpy()).copy()
    k = len(cols)
    L = A.copy()
    al = np.zeros(k, dtype=bool)
    for j in range(k):
        d = L[j, j]
        orig = Gn[cols[j], cols[j]]
        if not (orig > 0) or not (d > tol * tol * orig):
            al[j] = True
            L[j:, j] = 0.0
            continue
        ljj = np.sqrt(d)
        L[j + 1:, j] /= ljj
        L[j, j] = ljj
        L[j + 1:, j + 1:] -= np.tril(np.outer(L[j + 1:, j], L[j + 1:, j]))
    keep = ~al
    Lk = np.tril(L[np.ix_(keep, keep)])
    y = np.linalg.solve(Lk, b[keep]) if keep.any() else np.zeros(0)
    bk = np.linalg.solve(Lk.T, y) if keep.any() else np.zeros(0)
    beta = np.full(k, np.nan)
    beta[keep] = bk
    inv = np.full(k, np.nan)
    if keep.any():
        Linv = np.linalg.inv(Lk)
        inv[keep] = np.sum(Linv ** 2, axis=0)
    yty = Gn[rcol, rcol] if rcol >= 0 else 0.0
    aux = np.array([keep.sum(), yty - bk @ b[keep], yty, 0.0])
    dev = G.device
    return SolveResult(torch.from_numpy(beta).to(dev), torch.from_numpy(inv).to(dev),
                       torch.from_numpy(aux).to(dev))


def predict(panel: DevicePanel, cols, beta: torch.Tensor, override_idx: int = -1,
            override_val: float = 0.0, link: str = "identity",
            out: torch.Tensor | None = None) -> torch.Tensor:
    """eta = X[:, cols] beta (NaN beta = aliased -> 0); optional constant override of one
    design column (counterfactual W); link 'logit' applies the logistic function."""
    cols_t = cols if isinstance(cols, torch.Tensor) else const(cols, torch.int32, panel.device)
    lk = 1 if link == "logit" else 0
    if not panel.data.is_cuda:
        X = panel.data.double()[cols_t.long()].clone()
        if override_idx >= 0:
            X[override_idx] = override_val
        b = torch.nan_to_num(beta.double(), nan=0.0)
        eta = b @ X
        return logistic(eta) if lk else eta
    out = out if out is not None else torch.empty(panel.ld, dtype=torch.float64, device=panel.device)
    _native.call("ate_predict", dtype_code(panel.data), panel.data.data_ptr(), panel.cm_ld, panel.ld,
                 cols_t.data_ptr(), beta.data_ptr(), cols_t.numel(), override_idx, override_val, lk,
                 out.data_ptr(), _stream())
    return out


@dataclass
class IrlsResult:
    beta: torch.Tensor
    mu: torch.Tensor        # fitted probabilities (panel row order)
    eta: torch.Tensor
    state: torch.Tensor     # dev_old, dev, iters, converged
    done: torch.Tensor


def logistic_irls(panel: DevicePanel, cols, ycol: int, zcol: int, maxit: int = 25,
                  eps: float = 1e-8, dist=None) -> IrlsResult:
    """``glm(y ~ X[cols], binomial)`` by IRLS (glm.fit semantics: mustart=(y+.5)/2,
    |dev-dev_old|/(|dev|+0.1) < eps, maxit 25). GPU: fixed-budget launch sequence with
    a device convergence flag (no host sync; capturable in a hipGraph).

    ``dist`` (parallel.dist.DistContext): the panel is this rank's row shard; each
    iteration all-reduces the weighted Gram and the deviance partials (C01/C02), so
    every rank takes the same Newton step and the same convergence decision."""
    dev = panel.device
    cols_t = const(cols, torch.int32, dev)
    k = len(cols)
    if not panel.data.is_cuda:
        return _irls_cpu(panel, cols, ycol, zcol, maxit, eps, dist)
    nb = 1024
    eta = torch.empty(panel.ld, dtype=torch.float64, device=dev)
    mu = torch.empty_like(eta)
    w = torch.empty(panel.ld, dtype=panel.dtype, device=dev)
    devp = torch.empty(nb, dtype=torch.float64, device=dev)
    state = torch.zeros(4, dtype=torch.float64, device=dev)
    done = torch.zeros(1, dtype=torch.int32, device=dev)
    ws = SolveWorkspace(k, dev)
    dc = dtype_code(panel.data)
    s = _stream()
    X = panel.data
    _native.call("ate_irls_update", dc, X.data_ptr(), panel.cm_ld, panel.ld, cols_t.data_ptr(),
                 ws.beta.data_ptr(), k, ycol, panel.cols["one"], zcol, 1, eta.data_ptr(),
                 mu.data_ptr(), w.data_ptr(), devp.data_ptr(), nb, done.data_ptr(), s)
    if dist is not None:
        dist.sum_(devp)
    _native.call("ate_irls_check", devp.data_ptr(), nb, 1, eps, maxit, state.data_ptr(),
                 done.data_ptr(), s)
    Gsum = torch.empty((panel.P, panel.P), dtype=torch.float64, device=dev) if panel.nseg > 1 else None
    for _ in range(maxit):
        G = gram(panel, w, done=done)
        if Gsum is not None:
            torch.sum(G, dim=0, out=Gsum)
            G = Gsum
        else:
            G = G[0]
        if dist is not None:
            dist.sum_(G)
        chol_solve(G, cols_t, zcol, done=done, ws=ws)
        _native.call("ate_irls_update", dc, X.data_ptr(), panel.cm_ld, panel.ld, cols_t.data_ptr(),
                     ws.beta.data_ptr(), k, ycol, panel.cols["one"], zcol, 0, eta.data_ptr(),
                     mu.data_ptr(), w.data_ptr(), devp.data_ptr(), nb, done.data_ptr(), s)
        if dist is not None:
            dist.sum_(devp)
        _native.call("ate_irls_check", devp.data_ptr(), nb, 0, eps, maxit, state.data_ptr(),
                     done.data_ptr(), s)
    return IrlsResult(ws.beta, mu, eta, state, done)


def _binom_dev(y, mu):
    with np.errstate(divide="ignore", invalid="ignore"):
        t1 = np.where(y > 0, y * np.log(np.where(y > 0, y / mu, 1.0)), 0.0)
        t2 = np.where(y < 1, (1 - y) * np.log(np.where(y < 1, (1 - y) / (1 - mu), 1.0)), 0.0)
    return 2.0 * np.sum(t1 + t2)


def _irls_cpu(panel, cols, ycol, zcol, maxit, eps, dist=None):
    red = (lambda a: dist.sum_(torch.as_tensor(a, dtype=torch.float64)).numpy()) \
        if dist is not None else (lambda a: np.asarray(a, dtype=np.float64))
    X = panel.data.double().cpu().numpy()
    v = X[panel.cols["one"]] != 0
    A = X[cols][:, v]
    y = X[ycol, v]
    mu = (y + 0.5) / 2
    eta = np.log(mu / (1 - mu))
    dev_old = float(red([_binom_dev(y, mu)])[0])
    beta = np.zeros(len(cols))
    it = 0
    conv = False
    e10 = 10 * np.finfo(float).eps
    for it in range(1, maxit + 1):
        me = mu * (1 - mu)
        z = eta + (y - mu) / me
        G = (A * me) @ np.vstack([A, z]).T          # [k, k+1]
        Gfull = np.zeros((len(cols) + 1, len(cols) + 1))
        Gfull[:len(cols), :] = G
        Gfull[len(cols), :len(cols)] = G[:, len(cols)]
        Gfull[len(cols), len(cols)] = (me * z) @ z
        Gfull = red(Gfull)
        r = _chol_solve_cpu(torch.from_numpy(Gfull), np.arange(len(cols)), len(cols), None, LM_TOL)
        beta = r.beta.numpy()
        eta = np.nan_to_num(beta) @ A
        mu = np.clip(1 / (1 + np.exp(-eta)), e10, 1 - e10)
        dev = float(red([_binom_dev(y, mu)])[0])
        if abs(dev - dev_old) / (abs(dev) + 0.1) < eps:
            conv = True
            break
        dev_old = dev
    mu_full = np.zeros(panel.ld)
    eta_full = np.zeros(panel.ld)
    mu_full[v] = mu
    eta_full[v] = eta
    dev_ = panel.device
    return IrlsResult(torch.from_numpy(beta).to(dev_), torch.from_numpy(mu_full).to(dev_),
                      torch.from_numpy(eta_full).to(dev_),
                      torch.tensor([dev, dev, it, float(conv)], dtype=torch.float64),
                      torch.ones(1, dtype=torch.int32))
