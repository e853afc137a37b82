"""Forest engine (models/forest.py, csrc/cpu/forest_cpu.cpp) on the host.

R's randomForest/grf are not importable here, so exact parity with them is "unpinned":
these tests pin the engine's own contracts (determinism, thread-count invariance,
tree well-formedness, statistical sanity on signals with a known answer) and compare it
statistically with an INDEPENDENT implementation of the same Breiman semantics
(scikit-learn's RandomForestClassifier / Regressor). The GPU twins are checked against
this host engine bit-for-bit in tests/test_forest_gpu.py.
"""
import numpy as np
import pytest

from ate_replication_causalml_amd.models import forest as F


def _toy(n=3000, p=6, seed=0):
    r = np.random.default_rng(seed)
    X = r.normal(size=(n, p))
    X[:, 1] = np.round(X[:, 1])  # a few distinct values -> midpoint bins
    return X


def test_fixed_point_roundtrip():
    v = np.array([0.0, 1.0, -1.0, 0.123456789, -3.5e-6])
    back = F.from_fix(F.to_fix(v))
    assert np.max(np.abs(back - v)) <= 2.0 ** -32


def test_bin_edges_and_matrix():
    X = _toy()
    edges, ne = F.bin_edges(X)
    Xb = F.bin_matrix(X, (edges), ne).numpy()
    assert Xb.shape == (X.shape[1], X.shape[0])
    for j in range(X.shape[1]):
        e = edges[j, :ne[j]]
        assert np.all(np.diff(e) > 0)
        # bin b means edges[b-1] < x <= edges[b]
        expect = np.searchsorted(e, X[:, j], side="left")
        np.testing.assert_array_equal(Xb[j], expect)
    u = np.unique(X[:, 1])
    np.testing.assert_allclose(edges[1, :ne[1]], (u[1:] + u[:-1]) / 2)


def live_trees(fr):
    """Per-tree (feat, thr, left, val) restricted to the nodes actually grown."""
    feat, thr, left, val, nn = fr.tree_arrays()
    cap = fr.cap
    out = []
    for t in range(fr.params.ntree):
        s = slice(t * cap, t * cap + nn[t])
        out.append((feat[s], thr[s], left[s], val[s]))
    return nn, out


def assert_same_forest(a, b):
    na, ta = live_trees(a)
    nb, tb = live_trees(b)
    np.testing.assert_array_equal(na, nb)
    for x, y in zip(ta, tb):
        for u, v in zip(x, y):
            np.testing.assert_array_equal(u, v)
    np.testing.assert_array_equal(np.asarray(a.inbag if not hasattr(a.inbag, "cpu") else a.inbag.cpu()),
                                  np.asarray(b.inbag if not hasattr(b.inbag, "cpu") else b.inbag.cpu()))


def _tree_ok(fr):
    feat, thr, left, val, nn = fr.tree_arrays()
    cap = fr.cap
    for t in range(fr.params.ntree):
        m = nn[t]
        assert 1 <= m <= cap
        f = feat[t * cap:t * cap + m]
        lc = left[t * cap:t * cap + m]
        internal = f >= 0
        assert np.all(lc[internal] > 0) and np.all(lc[internal] + 1 < m)
        kids = np.concatenate([lc[internal], lc[internal] + 1])
        assert len(np.unique(kids)) == len(kids) == m - 1  # every node but the root once


def test_rf_classifier_deterministic_and_thread_invariant(monkeypatch):
    X = _toy()
    y = (X[:, 0] + 0.5 * X[:, 2] + np.random.default_rng(1).normal(size=len(X)) > 0).astype(float)
    monkeypatch.setenv("ATE_CPU_THREADS", "1")
    a = F.rf_classifier(X, y, num_trees=40, seed=7, backend="cpu")
    monkeypatch.setenv("ATE_CPU_THREADS", "8")
    b = F.rf_classifier(X, y, num_trees=40, seed=7, backend="cpu")
    assert_same_forest(a, b)
    _tree_ok(a)
    p = a.oob_proba()
    assert np.isnan(p).sum() < 0.01 * len(p)
    ok = ~np.isnan(p)
    acc = np.mean((p[ok] > 0.5) == (y[ok] > 0.5))
    assert acc > 0.7
    c = F.rf_classifier(X, y, num_trees=40, seed=8, backend="cpu")
    assert not np.array_equal(live_trees(a)[1][0][0], live_trees(c)[1][0][0])


def test_bootstrap_inbag_counts():
    X = _toy(n=1000)
    y = (X[:, 0] > 0).astype(float)
    fr = F.rf_classifier(X, y, num_trees=20, seed=3, backend="cpu")
    inbag = np.asarray(fr.inbag).reshape(20, 1000).astype(int)
    assert set(np.unique(inbag)) <= {0, 1}  # in-bag flags
    # n draws with replacement leave about e^-1 of the rows out of bag
    assert abs(np.mean(inbag == 0) - np.exp(-1)) < 0.03


def test_regression_forest_recovers_step():
    X = _toy(n=4000)
    r = np.random.default_rng(2)
    y = np.where(X[:, 0] > 0, 1.0, -1.0) + 0.3 * r.normal(size=len(X))
    fr = F.regression_forest(X, y, num_trees=100, seed=4, backend="cpu")
    _tree_ok(fr)
    pred = fr.predict_raw(None, oob=True)
    ok = ~np.isnan(pred)
    truth = np.where(X[:, 0] > 0, 1.0, -1.0)
    assert np.corrcoef(pred[ok], truth[ok])[0, 1] > 0.9
    # half-sampling: each tree holds sample_fraction * n rows in its subsample
    inbag = np.asarray(fr.inbag).reshape(100, -1)
    assert np.all(inbag.sum(1) == 2000)


def test_causal_forest_heterogeneous_effect():
    X = _toy(n=5000)
    r = np.random.default_rng(5)
    W = (r.uniform(size=len(X)) < 1 / (1 + np.exp(-0.5 * X[:, 2]))).astype(float)
    tau = 1.0 + (X[:, 0] > 0)
    Y = X[:, 2] + tau * W + 0.5 * r.normal(size=len(X))
    cf = F.causal_forest(X, Y, W, num_trees=200, seed=11, backend="cpu")
    est, se = F.average_treatment_effect(cf)
    assert abs(est - tau.mean()) < 4 * se + 0.05
    t = cf.tau_oob
    ok = ~np.isnan(t)
    assert np.corrcoef(t[ok], tau[ok])[0, 1] > 0.6
    assert np.all(cf.var_oob[ok] >= 0)
    assert 0.01 < np.sqrt(np.nanmean(cf.var_oob)) < 2.0


@pytest.mark.parametrize("splits", ["binned", "exact"])
def test_rf_oob_propensity_matches_sklearn_statistically(splits):
    """Independent cross-check of the randomForest semantics (ate_functions.R:169-174:
    bootstrap, mtry = floor(sqrt(p)), Gini, fully grown, OOB vote shares) against
    scikit-learn's RandomForestClassifier with the same settings on the tutorial DGP's
    selection-biased sample. Exact parity is impossible (different RNG, 256-bin vs exact
    thresholds); the OOB propensities must agree in distribution, discrimination (AUC)
    and calibration (Brier) within Monte Carlo error, and row by row (correlation)."""
    from sklearn.ensemble import RandomForestClassifier
    from sklearn.metrics import roc_auc_score
    from ate_replication_causalml_amd.data.dgp import make_tutorial_data
    from ate_replication_causalml_amd.data.selection import apply_selection_bias
    m, _ = apply_selection_bias(make_tutorial_data(30000, seed=1991))
    X, W = m.X, m.W
    ours = F.rf_classifier(X, W, num_trees=500, seed=7, backend="cpu", splits=splits).oob_proba()
    sk = RandomForestClassifier(n_estimators=500, max_features="sqrt", bootstrap=True,
                                min_samples_leaf=1, oob_score=True, random_state=0,
                                n_jobs=4).fit(X, W).oob_decision_function_[:, 1]
    ok = ~np.isnan(ours) & ~np.isnan(sk)
    assert ok.mean() > 0.99
    a, b, w = ours[ok], sk[ok], W[ok]
    assert abs(a.mean() - b.mean()) < 0.01
    assert abs(a.std() - b.std()) < 0.015
    assert abs(roc_auc_score(w, a) - roc_auc_score(w, b)) < 0.015
    assert abs(np.mean((a - w) ** 2) - np.mean((b - w) ** 2)) < 0.005
    # row by row: bounded by the OOB Monte Carlo noise (~184 OOB trees per row, sd ~0.03)
    # against the spread of the propensities on the calibrated DGP
    assert np.corrcoef(a, b)[0, 1] > 0.9
    np.testing.assert_allclose(np.quantile(a, [0.1, 0.5, 0.9]), np.quantile(b, [0.1, 0.5, 0.9]),
                               atol=0.02)


def test_rf_regressor_matches_sklearn_statistically():
    """Breiman regression forest (variance-reduction splits, leaf means, mtry = p/3)
    against scikit-learn's RandomForestRegressor: held-out R^2 and the predictions agree."""
    from sklearn.ensemble import RandomForestRegressor
    r = np.random.default_rng(3)
    n, p = 4000, 9
    X = r.normal(size=(n, p))
    y = np.sin(2 * X[:, 0]) + X[:, 1] * (X[:, 2] > 0) + 0.3 * r.normal(size=n)
    Xt = r.normal(size=(2000, p))
    yt = np.sin(2 * Xt[:, 0]) + Xt[:, 1] * (Xt[:, 2] > 0)
    ours = F.rf_regressor(X, y, num_trees=300, seed=4, backend="cpu").predict_proba(Xt)
    sk = RandomForestRegressor(n_estimators=300, max_features=1 / 3, min_samples_split=6,
                               random_state=0, n_jobs=4).fit(X, y).predict(Xt)
    r2 = lambda f: 1 - np.mean((f - yt) ** 2) / np.var(yt)
    assert abs(r2(ours) - r2(sk)) < 0.03 and r2(ours) > 0.7
    assert np.corrcoef(ours, sk)[0, 1] > 0.97


# ------------------------------------------------------------------ exact-split mode
def _exact_data(n=3000, p=6, seed=0, rounded=False):
    r = np.random.default_rng(seed)
    X = r.normal(size=(n, p))
    if rounded:
        X = np.round(X, 1)          # < 256 distinct values per feature
    W = (r.uniform(size=n) < 1 / (1 + np.exp(-X[:, 0] - X[:, 1] * X[:, 2]))).astype(float)
    Y = X[:, 1] + W * (1 + X[:, 0]) + 0.5 * r.normal(size=n)
    return X, W, Y


@pytest.mark.parametrize("kind", [F.KIND_CLASS, F.KIND_REG])
def test_exact_splits_equal_binned_engine_on_few_distinct_values(kind):
    """With <= 256 distinct values per feature the binned engine's bins are already the value
    ranks, so the sort-based exact engine must grow the same tree shapes (features, children,
    leaf values, in-bag rows); only thresholds may move inside the gap between a node's
    neighbouring values (binned: at the left value, exact: at the midpoint)."""
    X, W, Y = _exact_data(rounded=True)
    kw = dict(ntree=12, seed=5, backend="cpu")
    kw.update(y=W) if kind == F.KIND_CLASS else kw.update(r1=Y, min_node=5)
    a = F.fit_forest(X, kind, splits="exact", **kw)
    b = F.fit_forest(X, kind, **kw)
    fa, ta, la, va, na = a.tree_arrays()
    fb, tb, lb, vb, nb = b.tree_arrays()
    np.testing.assert_array_equal(na, nb)
    for t in range(12):
        s = slice(t * a.cap, t * a.cap + na[t])
        np.testing.assert_array_equal(fa[s], fb[s])
        np.testing.assert_array_equal(la[s], lb[s])
        np.testing.assert_array_equal(va[s], vb[s])
        assert (ta[s] >= tb[s]).all()
    np.testing.assert_array_equal(np.asarray(a.inbag), np.asarray(b.inbag))


def test_exact_split_thresholds_are_randomforest_midpoints():
    """Every split of an exact forest on continuous covariates sits at the midpoint of the
    node's two neighbouring in-bag values (randomForest findbestsplit): routing the in-bag
    rows down each tree, max(left values) <= thr value and the stored bin is the last table
    value <= (max left + min right) / 2."""
    X, W, _ = _exact_data(n=1500, p=5, seed=2)
    fr = F.fit_forest(X, F.KIND_CLASS, y=W, ntree=6, seed=9, backend="cpu", splits="exact")
    eb = fr.exact
    feat, thr, left, _, nn = fr.tree_arrays()
    inbag = np.asarray(fr.inbag).reshape(6, -1)
    checked = 0
    for t in range(6):
        base = t * fr.cap
        stack = [(0, np.flatnonzero(inbag[t]))]
        while stack:
            v, rows = stack.pop()
            f = feat[base + v]
            if f < 0:
                continue
            x = X[rows, f]
            go = fr.exact.bin(X[rows])[f] <= thr[base + v]
            lmax, rmin = x[go].max(), x[~go].min()
            mid = (lmax + rmin) / 2.0
            u = eb.vals[f, :eb.nval[f]]
            want = max(np.searchsorted(u, lmax), min(np.searchsorted(u, mid, side="right") - 1,
                                                     np.searchsorted(u, rmin) - 1))
            assert thr[base + v] == want
            checked += 1
            stack += [(left[base + v], rows[go]), (left[base + v] + 1, rows[~go])]
    assert checked > 500


def test_exact_splits_new_data_prediction_uses_midpoints():
    """Prediction on rows of the training table goes left iff value <= midpoint: a tree
    with one split on a single feature classifies a grid of table values accordingly."""
    x = np.array([0.0, 1.0, 4.0, 5.0] * 50)[:, None]
    y = (x[:, 0] > 2).astype(float)
    fr = F.fit_forest(x, F.KIND_CLASS, y=y, ntree=3, seed=1, backend="cpu", splits="exact")
    feat, thr, _, _, nn = fr.tree_arrays()
    assert (nn == 3).all() and (thr[::fr.cap] == 1).all()     # bins 0,1 | 2,3: at 2.5
    np.testing.assert_array_equal(fr.predict_proba(np.array([[0.0], [1.0], [4.0], [5.0]])),
                                  [0, 0, 1, 1])


def test_grf_exact_splits_use_the_left_value_as_threshold():
    """grf splits x <= v (the value itself), randomForest at the midpoint: a regression
    step between the table values 1 and 4 goes to bin 1 in both, but a NEW row x = 2.2
    (below the midpoint 2.5, above the value 1) goes left under randomForest and right
    under grf (ate_replication.Rmd:250: grf::causal_forest's orthogonalisation forests)."""
    x = np.array([0.0, 1.0, 4.0, 5.0] * 200)[:, None]
    y = np.where(x[:, 0] > 2, 1.0, 0.0)
    g = F.regression_forest(x, y, num_trees=8, seed=3, backend="cpu", splits="exact",
                            min_node=1, alpha=0.0)
    feat, thr, _, _, nn = g.tree_arrays()
    assert (thr[::g.cap][feat[::g.cap] >= 0] == 1).all()         # root split after value 1
    assert g.predict_proba(np.array([[2.2]]))[0] == pytest.approx(1.0)
    assert g.predict_proba(np.array([[0.5]]))[0] == pytest.approx(0.0)
    r = F.fit_forest(x, F.KIND_REG, r1=y, ntree=8, seed=3, backend="cpu", splits="exact")
    assert r.predict_proba(np.array([[2.2]]))[0] == pytest.approx(0.0)


def test_grf_sampling_little_bags_and_group_one():
    """grf's samples: with little bags (ci.group.size = 2) both trees of a group share the
    group's half-sample as in-bag rows; with ci.group.size = 1 (grf's Y.hat / W.hat
    forests) each tree's in-bag rows are its own floor(n * sample.fraction) subsample;
    with honesty the J2 half fills the estimation counts (root count = |J2|)."""
    r = np.random.default_rng(1)
    n = 2001
    X = r.normal(size=(n, 4))
    y = X[:, 0] + r.normal(size=n)
    g2 = F.fit_forest(X, F.KIND_REG, r1=y, ntree=4, sampling=1, honesty=True, group=2,
                      min_node=5, seed=7, backend="cpu", splits="exact")
    ib = np.asarray(g2.inbag).reshape(4, n)
    assert (ib.sum(1) == n // 2).all()
    np.testing.assert_array_equal(ib[0], ib[1])
    np.testing.assert_array_equal(ib[2], ib[3])
    assert (ib[0] != ib[2]).any()
    est = np.asarray(g2.est).reshape(4, g2.cap, 5)
    assert (est[:, 0, 0] == (n // 2) - (n // 2) // 2).all()      # J2 = |S| - |J1|
    g1 = F.fit_forest(X, F.KIND_REG, r1=y, ntree=4, sampling=1, honesty=True, group=1,
                      min_node=5, seed=7, backend="cpu", splits="exact")
    ib1 = np.asarray(g1.inbag).reshape(4, n)
    assert (ib1.sum(1) == n // 2).all() and (ib1[0] != ib1[1]).any()


def test_causal_forest_auto_uses_exact_splits_at_tutorial_scale():
    """causal_forest(splits="auto") grows grf's exact-split honest forests up to 65,536 rows
    (the exact engine's uint16 value ranks) and recovers a heterogeneous effect."""
    r = np.random.default_rng(5)
    n = 3000
    X = r.normal(size=(n, 5))
    W = (r.uniform(size=n) < 0.5).astype(float)
    tau = 1.0 + (X[:, 0] > 0)
    Y = X[:, 1] + tau * W + 0.3 * r.normal(size=n)
    cf = F.causal_forest(X, Y, W, num_trees=200, seed=3, backend="cpu")
    assert cf.forest.exact is not None and cf.forest.params.sampling == 1
    ate, se = F.average_treatment_effect(cf)
    assert abs(ate - tau.mean()) < 4 * se + 0.05
    hi, lo = cf.tau_oob[X[:, 0] > 0.5], cf.tau_oob[X[:, 0] < -0.5]
    assert np.nanmean(hi) - np.nanmean(lo) > 0.5


def test_aipw_average_effect_clipping_is_a_textbook_option():
    """grf's estimate_average_effect does not clip W.hat (it warns on poor overlap): the
    default reproduces that; clip= (compat="textbook" in the estimators) clips W.hat."""
    import warnings
    r = np.random.default_rng(2)
    n = 200
    W = (r.uniform(size=n) < 0.5).astype(float)
    Y = r.normal(size=n)
    w_hat = np.clip(r.uniform(0.2, 0.8, size=n), 0, 1)
    w_hat[0], W[0] = 1e-9, 1.0                       # one row with (almost) no overlap
    cf = F.CausalForestFit(None, np.zeros(n), w_hat, np.zeros(n), np.ones(n), Y, W)
    with warnings.catch_warnings(record=True) as rec:
        warnings.simplefilter("always")
        grf_est, _ = F.average_treatment_effect(cf)
    assert any("overlap" in str(x.message) for x in rec)
    tb_est, _ = F.average_treatment_effect(cf, clip=1e-6)
    # the unclipped score of row 0 is (1 - 1e-9) / 1e-9 * Y0 / n: ~1e6 / n
    assert abs(grf_est - tb_est) > 100 * abs(tb_est)
    w_c = np.clip(w_hat, 1e-6, 1 - 1e-6)
    g = (W - w_hat) / (w_c * (1 - w_c)) * Y
    assert np.isclose(tb_est, g.mean(), rtol=1e-12)


def test_auto_splits_bound_the_exact_list_scratch():
    """"auto" picks exact splits up to 65,536 rows only while a tree's two per-feature row
    lists (8 p n bytes) stay within EXACT_AUTO_LIST_BYTES: the tutorial's p = 21 keeps
    exact splits, a 512-column panel of 65,536 rows (268 MB of lists per tree) goes to the
    histogram engine; explicit choices are kept."""
    assert F.resolve_splits("auto", 9_416, 21) == "exact"
    assert F.resolve_splits("auto", 65_536, 128) == "exact"
    assert F.resolve_splits("auto", 65_536, 512) == "binned"
    assert F.resolve_splits("auto", 70_000, 5) == "binned"
    assert F.resolve_splits("auto", 65_536) == "exact"          # p unknown: rows only
    assert F.resolve_splits("exact", 65_536, 512) == "exact"
    assert F.exact_list_bytes(65_536, 512) == 268_435_456


def test_exact_overflow_flag_raises_at_first_host_read():
    """GPU exact-split fits keep the count of overflowed trees (nnodes = -1) on the device and
    Forest.check() raises at the first host read of the outputs (predict_raw, tree_arrays),
    so the fit itself never waits for the device; a clean count passes once and is dropped."""
    import dataclasses
    import torch
    rs = np.random.RandomState(0)
    X = rs.randn(300, 4)
    y = (X[:, 0] > 0).astype(float)
    fr = F.fit_forest(X, F.KIND_CLASS, y=y, ntree=4, seed=1, backend="cpu")
    bad = dataclasses.replace(fr, overflow=(torch.tensor(2), 4, 100))
    with pytest.raises(RuntimeError, match="2 of 4 trees overflowed"):
        bad.tree_arrays()
    assert bad.overflow is None
    ok = dataclasses.replace(fr, overflow=(torch.tensor(0), 4, 100))
    ok.tree_arrays()
    assert ok.overflow is None
