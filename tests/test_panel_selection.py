"""K04 at panel scale (data/panel_selection.py): the selection-bias transform over
generated rows keeps exactly N rows, equals the host transform of
``ate_replication.Rmd:97-121`` (data/selection.py) on the same rows, and gives the same
kept-row set at every world size (sharded candidate counting, kept-rank slices)."""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np
import pytest
import torch

from ate_replication_causalml_amd.data import dgp
from ate_replication_causalml_amd.data.device_dgp import fold_slices, synthetic_panel
from ate_replication_causalml_amd.data.panel_selection import (SEL_BR, kept_gids,
                                                                plan_selection)
from ate_replication_causalml_amd.data.selection import drop_indices
from ate_replication_causalml_amd.parallel.comm import run_simulated

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _host_kept(n_gen, seed, compat="reference"):
    """data/selection.py's transform of the first n_gen generated rows (raw = population-
    standardised yob / city)."""
    cts, binc, _, W, _, _ = dgp.raw_columns(n_gen, seed, params=dgp.TUTORIAL)
    X = np.column_stack([cts, binc])
    drop = drop_indices(X, W, dgp.COVARIATES, compat=compat)
    keep = np.ones(n_gen, dtype=bool)
    keep[drop] = False
    return np.flatnonzero(keep)


@pytest.mark.parametrize("n_keep,seed,compat", [(3000, 5, "reference"), (7001, 11, "reference"),
                                                (2500, 3, "textbook")])
def test_kept_rows_equal_host_transform(n_keep, seed, compat):
    sel = plan_selection(n_keep, seed, dgp.TUTORIAL, compat=compat)
    g = kept_gids(sel, [(0, n_keep)]).numpy()
    want = _host_kept(sel.n_gen, seed, compat)
    assert len(g) == n_keep == len(want)
    assert np.array_equal(g, want)
    # the n_gen-th generated row is the last one kept (n_gen is minimal)
    assert g[-1] == sel.n_gen - 1
    # the tutorial's scale: ~82 % of the generated rows dropped (41,062 of 50,000 published)
    assert 0.75 < 1 - n_keep / sel.n_gen < 0.88


def test_selection_spans_several_blocks():
    """N large enough that the transform runs over many SEL_BR blocks, with kept-rank
    slices that start and end inside blocks."""
    n = 9000
    sel = plan_selection(n, 2, dgp.TUTORIAL)
    assert sel.nblk >= 2 or sel.n_gen > SEL_BR // 2
    full = kept_gids(sel, [(0, n)]).numpy()
    parts = kept_gids(sel, [(17, 1000), (2000, 3), (4096, 4904)]).numpy()
    assert np.array_equal(parts, np.concatenate([full[17:1017], full[2000:2003], full[4096:]]))


@pytest.mark.parametrize("world", [2, 3, 4])
def test_kept_set_invariant_across_world_sizes(world):
    n, K = 4000, 5
    ref = kept_gids(plan_selection(n, 7, dgp.TUTORIAL), [(0, n)]).numpy()

    def rank_rows(comm):
        sel = plan_selection(n, 7, dgp.TUTORIAL, comm=comm)
        sl = fold_slices(n, K, comm.rank, comm.world_size)
        return sel, sl, kept_gids(sel, sl).numpy()

    outs = run_simulated(world, rank_rows)
    got = np.full(n, -1, dtype=np.int64)
    for sel, sl, g in outs:
        assert (sel.n_gen, sel.thr_t, sel.thr_c) == (outs[0][0].n_gen, outs[0][0].thr_t,
                                                     outs[0][0].thr_c)
        o = 0
        for a, c in sl:
            got[a:a + c] = g[o:o + c]
            o += c
    assert np.array_equal(got, ref)


def test_tutorial_panel_rows_invariant_across_ranks():
    """synthetic_panel(dgp="tutorial"): the rows of every rank's shard are the world-1 rows
    of the same kept ranks (CPU float64 panels)."""
    n, p = 2400, 24
    one = synthetic_panel(n, p=p, folds=5, seed=9, dtype="f64", device="cpu", dgp="tutorial")
    assert one.n == n and one.n_generated > n
    X1 = one.colmajor()

    def shard(comm):
        return synthetic_panel(n, p=p, folds=5, seed=9, dtype="f64", device="cpu",
                               dgp="tutorial", comm=comm)
    for pan in run_simulated(2, shard):
        m = pan.row_index >= 0
        rows = pan.row_index[m]
        pos1 = torch.nonzero(one.row_index >= 0).reshape(-1)
        # world-1 panel position of each kept rank
        where = torch.empty(n, dtype=torch.long)
        where[one.row_index[pos1]] = pos1
        assert torch.equal(pan.colmajor()[:, m], X1[:, where[rows]])


def test_tutorial_panel_is_confounded():
    """After selection W depends on the vote history (the RCT panel's W does not)."""
    pan = synthetic_panel(6000, p=21, folds=5, seed=4, dtype="f64", device="cpu", dgp="tutorial")
    rct = synthetic_panel(6000, p=21, folds=5, seed=4, dtype="f64", device="cpu", dgp="rct")

    def corr(pn):
        m = pn.row_index >= 0
        W = pn.col("W")[m]
        g2000 = pn.data[pn.cols["x16"]][m]          # first vote-history column
        return float(torch.corrcoef(torch.stack([W, g2000]))[0, 1])
    assert abs(corr(rct)) < 0.05
    # treated likely voters and control unlikely voters dropped: treated vote less
    assert corr(pan) < -0.1


def test_gloo_two_process_selection():
    """Real torch.distributed (gloo) ranks: sharded candidate counting, one all-reduce,
    every rank's kept-row slices equal the world-1 selection."""
    script = r"""
import os, sys, json
sys.path.insert(0, %r)
import torch, torch.distributed as dist
dist.init_process_group("gloo")
from ate_replication_causalml_amd.parallel.comm import TorchComm
from ate_replication_causalml_amd.data import dgp
from ate_replication_causalml_amd.data.device_dgp import fold_slices
from ate_replication_causalml_amd.data.panel_selection import plan_selection, kept_gids
c = TorchComm()
sel = plan_selection(5000, 13, dgp.TUTORIAL, comm=c)
sl = fold_slices(5000, 5, c.rank, c.world_size)
g = kept_gids(sel, sl).tolist()
out = [None] * c.world_size
dist.all_gather_object(out, [sel.n_gen, sl, g])
if c.rank == 0:
    print("RESULT", json.dumps(out))
dist.destroy_process_group()
""" % ROOT
    with tempfile.NamedTemporaryFile("w", suffix=".py", delete=False) as f:
        f.write(script)
        path = f.name
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", "--master-port=29533", path]
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=300)
    finally:
        os.unlink(path)
    assert r.returncode == 0, r.stderr[-3000:]
    outs = json.loads([l for l in r.stdout.splitlines() if l.startswith("RESULT")][0].split(" ", 1)[1])
    sel = plan_selection(5000, 13, dgp.TUTORIAL)
    ref = kept_gids(sel, [(0, 5000)]).numpy()
    got = np.full(5000, -1, dtype=np.int64)
    for n_gen, sl, g in outs:
        assert n_gen == sel.n_gen
        o = 0
        for a, c in sl:
            got[a:a + c] = g[o:o + c]
            o += c
    assert np.array_equal(got, ref)


def test_selected_rows_host_arrays():
    """data/panel_selection.selected_rows: the kept rows as host arrays (configs 3 / 4)."""
    from ate_replication_causalml_amd.data.panel_selection import selected_rows
    d, sel = selected_rows(2000, 4)
    assert d.X.shape == (2000, 21) and sel.n_gen > 2000
    g = kept_gids(sel, [(0, 2000)]).numpy()
    cts, binc, _, W, Y, _ = dgp.raw_columns(0, 4, params=dgp.TUTORIAL, idx=g)
    assert np.array_equal(d.X, np.column_stack([cts, binc])) and np.array_equal(d.W, W)


def test_emulated_comm_shapes():
    """parallel/comm.EmulatedComm (tools/cfg4.py / cfg5.py --shard r/W): rank r's share of
    every sharded algorithm, shape-correct non-communicating collectives."""
    from ate_replication_causalml_amd.parallel.comm import EmulatedComm
    c = EmulatedComm(2, 4)
    t = torch.arange(3.0)
    out = torch.empty(12)
    assert torch.equal(c.all_gather_into_(out, t), t.repeat(4))
    r = torch.empty(2)
    assert torch.equal(c.reduce_scatter_(r, torch.arange(8.0)), torch.tensor([4.0, 5.0]))
    assert len(c.all_gather(t)) == 4 and c.emulated
    with pytest.raises(ValueError):
        EmulatedComm(4, 4)


def test_plan_selection_rejects_degenerate_requests():
    from ate_replication_causalml_amd.data import panel_selection as PS
    from ate_replication_causalml_amd.data.dgp import TUTORIAL
    with pytest.raises(ValueError):
        PS.plan_selection(0, 1, TUTORIAL)
    with pytest.raises(ValueError):
        PS.plan_selection(10, 1, TUTORIAL, pt=0.0)
