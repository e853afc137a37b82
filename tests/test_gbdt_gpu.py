"""GPU GBDT kernels (csrc/gbdt.hip) vs the numpy reference: integer histograms and
IEEE-identical gains give the same trees."""
import numpy as np
import torch
import pytest

from ate_replication_causalml_amd.models import gbdt as G

from test_gbdt import _data

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("depth", [1, 3, 6, 8])
def test_gbdt_gpu_trees_identical_squared(gpu, depth):
    X, y = _data(5000, depth)
    tr = np.arange(len(y)) % 4 != 0
    edges = G.global_bin_edges(X, None)
    kw = dict(n_trees=6, depth=depth, lr=0.3, train=tr, edges=edges)
    a = G.fit_gbdt(X, y, backend="gpu", **kw)
    b = G.fit_gbdt(X, y, backend="cpu", **kw)
    np.testing.assert_array_equal(a.feat.cpu().numpy(), b.feat)
    np.testing.assert_array_equal(a.thr.cpu().numpy()[b.feat >= 0], b.thr[b.feat >= 0])
    np.testing.assert_allclose(a.value.cpu().numpy(), b.value, rtol=0, atol=0)
    np.testing.assert_allclose(a.predict(X), b.predict(X), rtol=1e-13, atol=1e-13)


def test_gbdt_gpu_logistic_close(gpu):
    X, y = _data(4000, 7)
    yb = (y > 0.3).astype(float)
    edges = G.global_bin_edges(X, None)
    kw = dict(loss="logistic", n_trees=8, depth=4, lr=0.3, edges=edges)
    a = G.fit_gbdt(X, yb, backend="gpu", **kw).predict(X, response=True)
    b = G.fit_gbdt(X, yb, backend="cpu", **kw).predict(X, response=True)
    # exp() may differ by an ulp between device and host libm -> fixed-point gradients can
    # differ by one unit; trees coincide except in exact near-ties
    assert np.mean(np.abs(a - b) < 1e-9) > 0.99


def test_dml_gbdt_gpu_vs_host(gpu, tutorial):
    from ate_replication_causalml_amd.estimators.boosting import dml_plr_gbdt
    _, m, _ = tutorial
    a = dml_plr_gbdt(m.Y, m.W, m.X, n_trees=10, depth=4, device=gpu)
    b = dml_plr_gbdt(m.Y, m.W, m.X, n_trees=10, depth=4, device="cpu")
    assert a.ate == pytest.approx(b.ate, abs=2e-3)
    assert a.se == pytest.approx(b.se, rel=0.05)


def _wide(n=20000, p=70, seed=3):
    r = np.random.default_rng(seed)
    X = r.normal(size=(n, p))
    X[:, 3] = np.round(X[:, 3])                 # a few-distinct-values feature
    y = np.sin(X[:, 0]) + 0.5 * (X[:, 40] > 0) + X[:, 69] * X[:, 3] + 0.1 * r.normal(size=n)
    return X, y


@pytest.mark.parametrize("sharded,depth", [(False, 6), (True, 6), (False, 8), (True, 8)])
def test_gbdt_gpu_wide_identical(gpu, sharded, depth):
    """p > 32 (several 32-feature histogram blocks, a partial last block), depth 6 / 8
    (five / seven partitions, up to 128 histogrammed nodes, histogram subtraction at every
    level); ``sharded`` runs the row-shard path (hessian child rule + reduce callback) on a
    one-rank context."""
    from ate_replication_causalml_amd.parallel.comm import LocalComm
    from ate_replication_causalml_amd.parallel.dist import DistContext
    X, y = _wide()
    tr = np.arange(len(y)) % 5 != 2
    edges = G.global_bin_edges(X, None)
    kw = dict(n_trees=4, depth=depth, lr=0.3, train=tr, edges=edges)
    dist = DistContext(LocalComm(), 0, len(y)) if sharded else None
    a = G.fit_gbdt(X, y, backend="gpu", dist=dist, **kw)
    b = G.fit_gbdt(X, y, backend="cpu", **kw)
    np.testing.assert_array_equal(a.feat.cpu().numpy(), b.feat)
    np.testing.assert_array_equal(a.thr.cpu().numpy()[b.feat >= 0], b.thr[b.feat >= 0])
    np.testing.assert_array_equal(a.value.cpu().numpy(), b.value)
    # scores of every row (train and held out) equal the host reference's
    np.testing.assert_allclose(a.scores.cpu().numpy(), b.scores, rtol=0, atol=1e-12)


def test_bin_edges_device_matches_host(gpu):
    import torch
    from ate_replication_causalml_amd.models import forest as F
    X, _ = _wide(5000, 70)
    e1, n1 = F.bin_edges(X)
    e2, n2 = F.bin_edges_device(torch.as_tensor(X, device=gpu))
    np.testing.assert_array_equal(n1, n2)
    np.testing.assert_array_equal(e1, e2)


@pytest.mark.parametrize("dtype", ["bf16", "f32"])
def test_bin_panel_matches_host_binning(gpu, dtype):
    # device binning of a resident panel == host binning of the same stored values
    from ate_replication_causalml_amd.data.device_dgp import synthetic_panel
    from ate_replication_causalml_amd.estimators.boosting import bin_panel
    from ate_replication_causalml_amd.models import forest as F
    pan = synthetic_panel(30011, p=40, folds=5, seed=5, dtype=dtype, device=gpu)
    Xr, ldr, edges, rows = bin_panel(pan)
    xc = torch.as_tensor(pan.xcols, device=gpu)
    Xh = pan.data.index_select(0, xc).index_select(1, rows).t().double().cpu().numpy()
    ref = F.bin_matrix(Xh, edges[0], edges[1], None).numpy()     # [p][n]
    assert Xr.shape[0] == len(rows) and ldr % 32 == 0
    assert np.array_equal(Xr[:, :40].t().cpu().numpy(), ref)
    assert int(Xr[:, 40:].max()) == 0


def test_dml_gbdt_panel_runs(gpu):
    from ate_replication_causalml_amd.data.device_dgp import synthetic_panel
    from ate_replication_causalml_amd.estimators.boosting import dml_plr_gbdt_panel
    pan = synthetic_panel(50000, p=30, folds=5, seed=9, dtype="bf16", device=gpu)
    r = dml_plr_gbdt_panel(pan, n_trees=20, depth=4)
    assert r.se > 0 and abs(r.ate - 0.09) < 0.06, r


def test_dml_gbdt_panel_dist_world1_equals_plain(gpu):
    """The row-sharded panel path (rule 1: pause per level, compact histogram all-reduce,
    here over a one-rank RCCL-free context) equals the single-device path bit for bit."""
    from ate_replication_causalml_amd.data.device_dgp import synthetic_panel
    from ate_replication_causalml_amd.estimators.boosting import dml_plr_gbdt_panel
    from ate_replication_causalml_amd.parallel.comm import LocalComm
    from ate_replication_causalml_amd.parallel.dist import DistContext
    pan = synthetic_panel(60000, p=37, folds=5, seed=9, dtype="bf16", device=gpu)
    a = dml_plr_gbdt_panel(pan, n_trees=6, depth=5)
    b = dml_plr_gbdt_panel(pan, n_trees=6, depth=5, dist=DistContext(LocalComm(), 0, pan.n))
    assert a.ate == b.ate and a.se == b.se


def test_dml_gbdt_panel_concurrent_pair_equals_serial(gpu):
    """A fold's E[Y|X] and E[W|X] fits on two streams (boosting._fit_pair) give the same
    bits as one after the other, with and without a (one-rank) row-sharded context."""
    from ate_replication_causalml_amd.data.device_dgp import synthetic_panel
    from ate_replication_causalml_amd.estimators.boosting import dml_plr_gbdt_panel
    from ate_replication_causalml_amd.parallel.comm import LocalComm
    from ate_replication_causalml_amd.parallel.dist import DistContext
    pan = synthetic_panel(60000, p=37, folds=5, seed=9, dtype="bf16", device=gpu)
    for dist in (None, DistContext(LocalComm(), 0, pan.n)):
        a = dml_plr_gbdt_panel(pan, n_trees=6, depth=5, dist=dist, concurrent=True)
        b = dml_plr_gbdt_panel(pan, n_trees=6, depth=5, dist=dist, concurrent=False)
        assert a.ate == b.ate and a.se == b.se


def test_dml_gbdt_panel_matches_host_arrays(gpu):
    """Panel path (device binning from the global sample, device Y/W/scores) == the
    host-array path on the same stored values (same edges: the full-data strided sample)."""
    from ate_replication_causalml_amd.data.device_dgp import synthetic_panel
    from ate_replication_causalml_amd.estimators.boosting import dml_plr_gbdt, dml_plr_gbdt_panel
    pan = synthetic_panel(40000, p=25, folds=5, seed=4, dtype="f32", device=gpu)
    a = dml_plr_gbdt_panel(pan, n_trees=5, depth=4)
    rows = torch.cat([torch.arange(int(s0), int(s0) + int(c), device=gpu)
                      for (s0, _), c in zip(pan.seg_bounds, pan.seg_nreal)])
    xc = torch.as_tensor(pan.xcols, device=gpu)
    X = pan.data.index_select(0, xc).index_select(1, rows).t().double().cpu().numpy()
    Y = pan.col("Y")[rows].double().cpu().numpy()
    W = pan.col("W")[rows].double().cpu().numpy()
    fid = np.repeat(np.arange(5), np.asarray(pan.seg_nreal))
    import ate_replication_causalml_amd.parallel.rng as R
    orig = R.fold_ids
    try:
        R.fold_ids = lambda n, K, seed, stream: fid      # the panel's fold = its segment
        b = dml_plr_gbdt(Y, W, X, n_trees=5, depth=4, device=gpu)
    finally:
        R.fold_ids = orig
    assert a.ate == pytest.approx(b.ate, abs=1e-12) and a.se == pytest.approx(b.se, rel=1e-10)


@pytest.mark.parametrize("mode", ["single", "world1", "sliced", "ranges"])
def test_gbdt_pair_fused_root_equals_two_fits(gpu, mode):
    """fit_gbdt_pair (a fold's two fits in lockstep, level 0 of both from ONE fused
    four-channel histogram pass, csrc/gbdt.hip gbdt_hist2_kernel) grows the trees of two
    fit_gbdt calls bit for bit: squared + logistic targets, p = 70 (a partial 16-feature
    block), depth 6; single device (rule 0), a one-rank row-sharded context (rule 1, root
    histogram all-reduced) and an emulated rank 0 of 2 (feature-sliced C04: root histogram
    reduce-scattered); "ranges": training rows in two runs (a fold's complement), the
    variant that computes each position's row instead of loading it."""
    from ate_replication_causalml_amd.parallel.comm import EmulatedComm, LocalComm
    from ate_replication_causalml_amd.parallel.dist import DistContext
    X, y = _wide()
    yb = (y > 0.4).astype(float)
    r = np.arange(len(y))
    tr = torch.as_tensor((r < 5000) | (r >= 9000) if mode == "ranges" else r % 5 != 2,
                         device=gpu)
    assert (G._two_ranges(torch.nonzero(tr).flatten().to(torch.int32))[1] >= 0) == (mode == "ranges")
    edges = G.global_bin_edges(X, None)
    Xb = G.binned(X, edges, gpu)
    dist = {"single": None, "world1": DistContext(LocalComm(), 0, len(y)),
            "sliced": DistContext(EmulatedComm(0, 2), 0, len(y)), "ranges": None}[mode]
    ty = torch.as_tensor(y, device=gpu)
    tw = torch.as_tensor(yb, device=gpu)
    kw = dict(n_trees=5, depth=6, lr=0.3)
    pa, pb = G.fit_gbdt_pair([ty, tw], ["squared", "logistic"], tr, Xb, edges, dist=dist, **kw)
    sa = G.fit_gbdt(None, ty, loss="squared", train=tr, dist=dist, edges=edges, Xb=Xb, **kw)
    sb = G.fit_gbdt(None, tw, loss="logistic", train=tr, dist=dist, edges=edges, Xb=Xb, **kw)
    for p_, s_ in ((pa, sa), (pb, sb)):
        assert torch.equal(p_.feat, s_.feat) and torch.equal(p_.thr, s_.thr)
        assert torch.equal(p_.value, s_.value) and torch.equal(p_.scores, s_.scores)
        assert int((p_.feat >= 0).sum()) > 20


def test_dml_gbdt_panel_fused_root_same_bits(gpu, monkeypatch):
    """The config-5 cross-fit with the fused root pass (the default) and with the two fits
    of a fold one after the other (ATE_GBDT_FUSED_ROOT=0): the same ATE/SE bits."""
    from ate_replication_causalml_amd.data.device_dgp import synthetic_panel
    from ate_replication_causalml_amd.estimators.boosting import dml_plr_gbdt_panel
    pan = synthetic_panel(60000, p=37, folds=5, seed=9, dtype="bf16", device=gpu,
                          dgp="tutorial")
    a = dml_plr_gbdt_panel(pan, n_trees=6, depth=5)
    monkeypatch.setattr(G, "FUSED_ROOT", False)
    b = dml_plr_gbdt_panel(pan, n_trees=6, depth=5)
    assert a.ate == b.ate and a.se == b.se
