"""HBM-resident design panel.

Layout: column-major ``data[P, ld]`` (one contiguous row vector per column, so a
16-byte load covers 8 consecutive rows of one column — the MFMA fragment shape
of the Gram kernel), rows grouped **fold-contiguously**: segment s (cross-fit
fold) occupies rows [seg_start[s], seg_end[s]) and is zero-padded to a multiple
of the Gram K-step. Zero rows contribute nothing to any Gram, and the ``one``
column doubles as the row-validity mask.

Standard columns: ``one`` (1 on real rows), covariates ``x0..x{p-1}``, ``W``,
``Y``, optional scratch columns (IRLS working response ``z``...). For bf16
panels, W and Y are also stored split as hi+lo bf16 pairs so X'W and X'Y
come out of the bf16 Gram at ~16-bit precision (exact for binary W, Y).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np
import torch

ROW_ALIGN = 64  # Gram K-step (bf16 kernel); also a multiple of the fp32/fp64 K-step (16)


def _dtype(name):
    return {"bf16": torch.bfloat16, "f32": torch.float32, "f64": torch.float64}[name]


def dtype_code(t: torch.Tensor) -> int:
    return {torch.float32: 1, torch.float64: 2, torch.bfloat16: 3}[t.dtype]


@dataclass
class DevicePanel:
    data: torch.Tensor                 # [P, ld]
    n: int                             # real rows
    cols: dict                         # name -> column index
    seg_bounds: np.ndarray             # (nseg, 2) padded row ranges
    seg_nreal: np.ndarray              # (nseg,) real rows per segment
    row_index: torch.Tensor            # (ld,) original row id (-1 on padding)
    xcols: list = field(default_factory=list)
    identity: bool = False             # real rows are rows 0..n-1 in order (one segment)
    # 64-row blocked layout: data is [ld/64, P, 64], element (c, i) at
    # (i/64)*64*P + c*64 + i%64. One Gram K-step (64 rows x all P columns) is then one
    # contiguous 64*P*2-byte run of HBM instead of P runs of 128 bytes ld apart
    # (profiles/r01_pmc/gram_diag.txt). Kernels that take (cs, bs) strides read both
    # layouts; the others require column-major (``cm_ld`` raises).
    blocked: bool = False
    # exact (world-size-invariant) Gram: rows of every segment form blocks of this many
    # rows counted from the segment start, the same blocks at every world size
    # (data/device_dgp.fold_slices(align=...)); 0 = not block-aligned
    exact_block: int = 0
    # one-byte copy of physical columns 384..P-1 when they are all {0, 1}-valued (P = 512
    # blocked bf16 panels from data/device_dgp.synthetic_panel): [ld/64, 128, 64] uint8, 0x3F
    # for 1; the paired-tile Gram streams it instead of those bf16 columns (csrc/gram.hip)
    bytes8: torch.Tensor | None = None

    @property
    def P(self):
        return self.data.shape[1] if self.blocked else self.data.shape[0]

    @property
    def ld(self):
        """Padded row count (and the column stride of a column-major panel)."""
        return self.data.shape[0] * ROW_ALIGN if self.blocked else self.data.shape[1]

    @property
    def cm_ld(self):
        """Leading dimension for kernels that only read column-major panels."""
        if self.blocked:
            raise NotImplementedError("this kernel reads column-major panels only; build the "
                                      "panel with blocked=False")
        return self.data.shape[1]

    def strides(self):
        """(cs, bs): element (c, i) at c*cs + (i/64)*bs + i%64."""
        return (ROW_ALIGN, ROW_ALIGN * self.P) if self.blocked else (self.ld, ROW_ALIGN)

    @property
    def device(self):
        return self.data.device

    @property
    def dtype(self):
        return self.data.dtype

    @property
    def nseg(self):
        return len(self.seg_bounds)

    def col(self, name) -> torch.Tensor:
        c = self.cols[name]
        return self.data[:, c, :].reshape(-1) if self.blocked else self.data[c]

    def valid(self) -> torch.Tensor:
        return self.col("one")

    def colmajor(self) -> torch.Tensor:
        """[P, ld] column-major view (a copy for a blocked panel)."""
        if not self.blocked:
            return self.data
        return self.data.permute(1, 0, 2).reshape(self.P, self.ld)

    def gather_rows(self, v: torch.Tensor) -> torch.Tensor:
        """Map a per-original-row vector into panel row order (0 on padding)."""
        out = torch.zeros(self.ld, dtype=v.dtype, device=self.device)
        if self.identity:                 # no mask indexing: no host sync, capturable
            out[:self.n] = v.to(self.device)
            return out
        m = self.row_index >= 0
        out[m] = v.to(self.device)[self.row_index[m]]
        return out

    def scatter_rows(self, v: torch.Tensor) -> torch.Tensor:
        """Map a panel-ordered vector (rows on dim 0) back to original row order."""
        if self.identity:
            return v[:self.n].clone()
        m = self.row_index >= 0
        out = torch.empty((self.n,) + tuple(v.shape[1:]), dtype=v.dtype, device=v.device)
        out[self.row_index[m]] = v[m]
        return out


def _round_up(x, m):
    return (x + m - 1) // m * m


def build_panel(X, W=None, Y=None, folds=None, dtype="f64", device="cpu", extra_cols=(),
                col_align=None, split_hi_lo=None) -> DevicePanel:
    """Assemble a panel from host arrays.

    folds: optional (n,) int fold id -> one padded segment per fold (in fold order).
    extra_cols: names of zero-initialised scratch columns to reserve.
    X may be a torch tensor (e.g. already in HBM): its fold gather and transposition
    then run on ``device`` (no host round trip of the n x p block); same values.
    """
    Xt = None
    if isinstance(X, torch.Tensor):
        Xt = X.to(device=device, dtype=torch.float64)
        if Xt.ndim == 1:
            Xt = Xt[:, None]
        X = np.empty(tuple(Xt.shape), dtype=np.float64)     # shape only
    X = np.asarray(X, dtype=np.float64)
    if X.ndim == 1:
        X = X[:, None]
    n, p = X.shape
    tdt = _dtype(dtype)
    if split_hi_lo is None:
        split_hi_lo = dtype == "bf16"
    if col_align is None:
        col_align = 128 if dtype == "bf16" else 64
    names = ["one"] + [f"x{j}" for j in range(p)]
    vecs = {}
    if W is not None:
        names.append("W")
        vecs["W"] = np.asarray(W, float)
    if Y is not None:
        names.append("Y")
        vecs["Y"] = np.asarray(Y, float)
    if split_hi_lo:
        for k in list(vecs):
            names += [f"{k}_hi", f"{k}_lo"]
    names += list(extra_cols)
    P = _round_up(len(names), col_align)
    if folds is None:
        folds = np.zeros(n, dtype=np.int64)
    folds = np.asarray(folds, dtype=np.int64)
    K = int(folds.max()) + 1 if n else 1
    order = np.argsort(folds, kind="stable")
    counts = np.bincount(folds, minlength=K)
    padded = np.array([_round_up(max(c, 1), ROW_ALIGN) for c in counts])
    starts = np.concatenate([[0], np.cumsum(padded)[:-1]])
    ld = int(padded.sum())
    row_index = np.full(ld, -1, dtype=np.int64)
    pos = 0
    for k in range(K):
        rows = order[pos:pos + counts[k]]
        row_index[starts[k]:starts[k] + counts[k]] = rows
        pos += counts[k]
    m = row_index >= 0
    ri = row_index[m]
    # host rows: everything but the x block when X is on the device
    host = np.zeros((P if Xt is None else P - p, ld), dtype=np.float64)
    hrow = (lambda r: r) if Xt is None else (lambda r: r if r == 0 else r - p)
    host[0, m] = 1.0
    if Xt is None:
        host[1:1 + p, m] = X[ri].T
    c = 1 + p
    cols = {n_: i for i, n_ in enumerate(names)}
    for k, v in vecs.items():
        host[hrow(cols[k]), m] = v[ri]
    if split_hi_lo:
        for k, v in vecs.items():
            hi = torch.from_numpy(v[ri]).to(torch.bfloat16).double().numpy()
            lo = v[ri] - hi
            host[hrow(cols[f"{k}_hi"]), m] = hi
            host[hrow(cols[f"{k}_lo"]), m] = lo
    if Xt is None:
        data = torch.from_numpy(host).to(tdt).to(device)
    else:
        data = torch.empty((P, ld), dtype=tdt, device=device)
        rest = torch.from_numpy(host).to(tdt).to(device)
        data[:1] = rest[:1]
        data[1 + p:] = rest[1:]
        blk = torch.zeros((p, ld), dtype=torch.float64, device=device)
        blk[:, torch.from_numpy(np.flatnonzero(m)).to(device)] = \
            Xt[torch.from_numpy(ri).to(device)].T
        data[1:1 + p] = blk.to(tdt)
    seg_bounds = np.stack([starts, starts + padded], axis=1)
    return DevicePanel(data=data, n=n, cols=cols, seg_bounds=seg_bounds,
                       seg_nreal=counts.astype(np.int64),
                       row_index=torch.from_numpy(row_index).to(device),
                       xcols=[cols[f"x{j}"] for j in range(p)], identity=K == 1)


def empty_panel(n_per_seg, P, dtype="bf16", device="cpu", blocked=False):
    """Allocate a panel with the given real rows per segment (filled later on device)."""
    counts = np.asarray(n_per_seg, dtype=np.int64)
    padded = np.array([_round_up(max(int(c), 1), ROW_ALIGN) for c in counts])
    starts = np.concatenate([[0], np.cumsum(padded)[:-1]])
    ld = int(padded.sum())
    shape = (ld // ROW_ALIGN, P, ROW_ALIGN) if blocked else (P, ld)
    data = torch.zeros(shape, dtype=_dtype(dtype), device=device)
    row_index = torch.full((ld,), -1, dtype=torch.int64, device=device)
    base = 0
    for s, c in zip(starts, counts):
        row_index[s:s + c] = torch.arange(base, base + c, device=device)
        base += int(c)
    return DevicePanel(data=data, n=int(counts.sum()), cols={"one": 0},
                       seg_bounds=np.stack([starts, starts + padded], axis=1),
                       seg_nreal=counts, row_index=row_index, identity=len(counts) == 1,
                       blocked=blocked)
