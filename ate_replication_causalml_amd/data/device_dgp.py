"""Synthetic tutorial-shape panels generated directly on the device (K-fold,
row-sharded across ranks) for the scaled configs (N = 1e6 .. 1e8, p = 21 .. 2000).

Global row g belongs to fold ``g * K // N``; rank r of R holds the r-th contiguous
slice of every fold. Rows are a pure function of (seed, g) (``csrc/dgp.hip``), so
the union of all shards is the same data set for every world size.

Two data-generating processes (``dgp=``):

* ``"tutorial"`` -- the tutorial's ``df_mod`` at scale: the calibrated
  latent-voter model (dgp.TUTORIAL) drawn as an RCT, then the selection-bias transform of
  ``ate_replication.Rmd:97-121`` over the generated rows (data/panel_selection.py): the
  first round(0.85 k) treated likely voters and control unlikely voters in generated-row
  order are dropped, and exactly N rows are kept (``n_generated`` records how many were
  drawn). W is confounded with the vote history, yob and city; "row g" above is then the
  g-th KEPT row.
* ``"tutorial-rct"`` -- the same calibrated model WITHOUT the transform: the tutorial's
  unbiased ``df`` at scale (its naive difference in means is the "oracle" row).
* ``"rct"`` -- the survey's scratch panel constants (dgp.PANEL) without selection: W is
  independent of X (a pure RCT), the path solver's worst case (every coordinate of the W
  nuisance is noise).
"""
from __future__ import annotations

import os

import numpy as np
import torch

from .. import _native
from ..ops.panel import DevicePanel, empty_panel, dtype_code
from . import dgp as host_dgp

N_TUTORIAL_COLS = 21
DGPS = ("tutorial", "tutorial-rct", "rct")


def fold_slices(n_total: int, folds: int, rank: int = 0, world: int = 1, align: int = 0):
    """[(global_start, count)] of this rank's slice of each fold. ``align`` > 0: slices are
    cut at multiples of ``align`` rows from the fold start (whole blocks per rank), the
    layout of the world-size-invariant exact reduction mode (ops/gram.py ``exact``)."""
    out = []
    for k in range(folds):
        f0, f1 = k * n_total // folds, (k + 1) * n_total // folds
        m = f1 - f0
        if align:
            nb = -(-m // align)
            a = min(f1, f0 + (rank * nb // world) * align)
            b = min(f1, f0 + ((rank + 1) * nb // world) * align)
        else:
            a = f0 + rank * m // world
            b = f0 + (rank + 1) * m // world
        out.append((a, b - a))
    return out


# One-byte columns (csrc/gram.hip, the paired-tile Gram's byte path): a P = 512 blocked bf16
# panel on the GPU keeps its {0, 1}-valued columns (one, the 6 tutorial binaries, every 4th
# extra covariate, W, Y and their hi / lo halves, padding) in physical columns 384..511 and a
# one-byte copy of those 128 columns beside the panel (DevicePanel.bytes8). Estimators see
# the same names -> columns map (pan.cols / pan.xcols); the Gram streams 896 instead of
# 1,024 bytes per row (profiles/r06_gram/README.md: 4.47 vs 4.54 ms per ate_dml call, the
# same bits). ATE_PANEL_BYTES=0: the generator's column order, no byte copy.
BYTE_COL0 = 384
BYTE_PANEL = os.environ.get("ATE_PANEL_BYTES", "1") == "1"


def _binary_names(p: int) -> set:
    """Generator columns whose values are exactly 0 or 1 (csrc/dgp.hip dgp_fill_kernel)."""
    out = {"one", "W", "Y", "W_hi", "W_lo", "Y_hi", "Y_lo"}
    out |= {f"x{j}" for j in range(15, min(21, p))}                    # sex + vote history
    out |= {f"x{j}" for j in range(21, p) if (j - 21) % 4 == 3}        # binary extras
    return out


def byte_column_order(names: list, p: int, P: int):
    """Physical column order for the one-byte path: the continuous columns first, then the
    binary ones, so that physical columns BYTE_COL0..P-1 are all binary or padding. None
    when the panel does not have that shape (P != 512, or too few binary columns)."""
    if P != 512:
        return None
    binary = _binary_names(p)
    cont = [nm for nm in names if nm not in binary]
    if len(cont) > BYTE_COL0:
        return None
    return cont + [nm for nm in names if nm in binary]


def synthetic_panel(n_total: int, p: int = 500, folds: int = 5, seed: int = 1991,
                    dtype: str = "bf16", device="cpu", rank: int = 0, world: int = 1,
                    blocked: bool = False, align: int = 0, dgp: str = "rct", comm=None,
                    selection=None, compat: str = "reference") -> DevicePanel:
    """``align`` > 0: block-aligned rank slices (fold_slices); the panel then records
    ``exact_block`` = align, the row block of the exact (world-size-invariant) Gram.

    ``dgp="tutorial"``: ``n_total`` rows are KEPT by the selection transform; ``comm``
    shards its candidate counting over the ranks (one all-reduce of per-block counts);
    ``selection``: a PanelSelection already planned for these (n_total, seed) (e.g. by the
    bf16 panel, reused for its float64 parity twin). The panel records ``dgp``,
    ``n_generated`` and ``selection``."""
    if p < N_TUTORIAL_COLS:
        raise ValueError("p must be >= 21 (tutorial columns)")
    if dgp not in DGPS:
        raise ValueError(f"dgp must be one of {DGPS}, got {dgp!r}")
    if comm is not None:
        rank, world = comm.rank, comm.world_size
    p_extra = p - N_TUTORIAL_COLS
    params = host_dgp.PANEL if dgp == "rct" else host_dgp.TUTORIAL
    slices = fold_slices(n_total, folds, rank, world, align)
    hi_lo = dtype == "bf16"
    names = ["one"] + [f"x{j}" for j in range(p)] + ["W", "Y"]
    if hi_lo:
        names += ["W_hi", "W_lo", "Y_hi", "Y_lo"]
    cpad = 128 if dtype == "bf16" else 64
    P = (len(names) + cpad - 1) // cpad * cpad
    pan = empty_panel([c for _, c in slices], P, dtype=dtype, device=device, blocked=blocked)
    order = byte_column_order(names, p, P) if (
        hi_lo and blocked and pan.data.is_cuda and BYTE_PANEL) else None
    pan.cols = {nm: i for i, nm in enumerate(names if order is None else order)}
    pan.xcols = [pan.cols[f"x{j}"] for j in range(p)]
    pcol = None
    if order is not None:
        pcol = torch.as_tensor([pan.cols[nm] for nm in names], dtype=torch.int16,
                               device=pan.data.device)
        pan.bytes8 = torch.zeros((pan.ld // 64, P - BYTE_COL0, 64), dtype=torch.uint8,
                                 device=pan.data.device)
    # global (kept) row ids of this shard (panel order)
    rid = torch.full((pan.ld,), -1, dtype=torch.int64, device=device)
    for (g0, cnt), (r0, _) in zip(slices, pan.seg_bounds):
        rid[r0:r0 + cnt] = torch.arange(g0, g0 + cnt, device=device)
    pan.row_index = rid
    pan.identity = len(slices) == 1 and slices[0][0] == 0
    gids = None
    sel = None
    if dgp == "tutorial":
        from .panel_selection import kept_gids, plan_selection
        pcomm = None if getattr(comm, "emulated", False) else comm   # --shard r/W: plan alone
        sel = selection if selection is not None else plan_selection(
            n_total, seed, params, comm=pcomm, device=pan.data.device, compat=compat)
        if sel.n_keep != n_total or sel.seed != seed:
            raise ValueError("selection plan does not match (n_total, seed)")
        if sel.compat != compat or sel.params != params:
            raise ValueError(f"selection plan made for compat={sel.compat!r} / other DGP "
                             f"parameters, not compat={compat!r}")
        gids = kept_gids(sel, slices, device=pan.data.device)
    offs = np.concatenate([[0], np.cumsum([c for _, c in slices])])
    if pan.data.is_cuda:
        s = torch.cuda.current_stream().cuda_stream
        pblk = np.ascontiguousarray(params.device_block())
        for k, ((g0, cnt), (r0, _)) in enumerate(zip(slices, pan.seg_bounds)):
            gp = 0 if gids is None or cnt == 0 else gids[int(offs[k]):].data_ptr()
            _native.call("ate_dgp_fill", dtype_code(pan.data), pan.data.data_ptr(),
                         *pan.strides(), int(r0), cnt, g0, gp, seed, p_extra, int(hi_lo),
                         pblk.ctypes.data, None if pcol is None else pcol.data_ptr(),
                         None if pcol is None else pan.bytes8.data_ptr(), s)
    else:
        cm = torch.zeros((pan.P, pan.ld), dtype=pan.data.dtype) if blocked else pan.data
        for k, ((g0, cnt), (r0, _)) in enumerate(zip(slices, pan.seg_bounds)):
            idx = None if gids is None else gids[int(offs[k]):int(offs[k]) + cnt].numpy()
            cts, binc, extra, W, Y, _ = host_dgp.raw_columns(cnt, seed, p_extra, row_offset=g0,
                                                              params=params, idx=idx)
            cols = [np.ones(cnt), *cts.T, *binc.T, *extra.T, W, Y]
            if hi_lo:
                cols += [W, np.zeros(cnt), Y, np.zeros(cnt)]
            block = torch.from_numpy(np.stack(cols)).to(pan.data.dtype)
            cm[:block.shape[0], r0:r0 + cnt] = block
        if blocked:
            pan.data.copy_(cm.reshape(pan.P, -1, 64).permute(1, 0, 2))
    pan.n = sum(c for _, c in slices)
    pan.exact_block = int(align)
    pan.dgp = dgp
    pan.selection = sel
    pan.n_generated = sel.n_gen if sel is not None else n_total
    pan.gen_ids = gids
    return pan
