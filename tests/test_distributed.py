"""Row-sharded (data-parallel) estimators: simulated worlds of 2 and 3 ranks
(in-process ThreadSimComm, rank-ordered reductions) must reproduce the single-device
results — the GLM/LASSO/AIPW paths all-reduce sufficient statistics (C01/C02/C06),
CV folds use global Philox fold ids, bootstrap replicates are sharded (C07)."""
import numpy as np
import pytest
import torch

from ate_replication_causalml_amd.estimators import lasso as DL
from ate_replication_causalml_amd.estimators import linear as D
from ate_replication_causalml_amd.parallel.comm import run_simulated
from ate_replication_causalml_amd.parallel.dist import DistContext, shard_range


def _run(fn, world, n):
    def body(comm):
        dist = DistContext.for_rank(comm, n)
        return fn(dist)
    return run_simulated(world, body)


def test_shard_range_partitions():
    for n, w in [(10, 3), (7, 4), (100, 8)]:
        got = [shard_range(n, r, w) for r in range(w)]
        assert got[0][0] == 0 and sum(c for _, c in got) == n
        assert all(got[i][0] + got[i][1] == got[i + 1][0] for i in range(w - 1))


@pytest.mark.parametrize("world", [2, 3])
def test_glm_family_sharded_equals_single(tutorial, world):
    _, m, _ = tutorial
    Y, W, X = m.Y, m.W, m.X
    n = len(Y)
    p1 = D.propensity_logistic(W, X, device="cpu").numpy()
    single = {
        "naive": D.naive(Y, W, device="cpu"),
        "ols": D.ols(Y, W, X, device="cpu"),
        "ipw": D.ipw(Y, W, X, p1, device="cpu"),
        "wls": D.ipw_wls(Y, W, p1, device="cpu"),
        "aipw": D.aipw_glm(Y, W, X, device="cpu"),
        "aipw_boot": D.aipw_glm(Y, W, X, bootstrap_se=True, B=40, device="cpu"),
    }

    def fn(dist):
        y, w, x = dist.local(Y), dist.local(W), dist.local(X)
        pl = D.propensity_logistic(w, x, device="cpu", dist=dist).numpy()
        return {
            "p": pl,
            "naive": D.naive(y, w, device="cpu", dist=dist),
            "ols": D.ols(y, w, x, device="cpu", dist=dist),
            "ipw": D.ipw(y, w, x, pl, device="cpu", dist=dist),
            "wls": D.ipw_wls(y, w, pl, device="cpu", dist=dist),
            "aipw": D.aipw_glm(y, w, x, device="cpu", dist=dist),
            "aipw_boot": D.aipw_glm(y, w, x, bootstrap_se=True, B=40, device="cpu", dist=dist),
        }

    outs = _run(fn, world, n)
    np.testing.assert_allclose(np.concatenate([o["p"] for o in outs]), p1, rtol=1e-10, atol=1e-12)
    for k, ref in single.items():
        for o in outs:
            assert o[k].ate == pytest.approx(ref.ate, rel=1e-9, abs=1e-12), k
            assert o[k].se == pytest.approx(ref.se, rel=1e-8, abs=1e-12), k


@pytest.mark.parametrize("world", [2, 3])
def test_lasso_family_sharded_equals_single(tutorial, world):
    _, m, _ = tutorial
    Y, W, X = m.Y, m.W, m.X
    n = len(Y)
    single = [DL.lasso_single(Y, W, X, device="cpu"), DL.lasso_usual(Y, W, X, device="cpu"),
              DL.dml_plr_lasso(Y, W, X, device="cpu")]

    def fn(dist):
        y, w, x = dist.local(Y), dist.local(W), dist.local(X)
        return [DL.lasso_single(y, w, x, device="cpu", dist=dist),
                DL.lasso_usual(y, w, x, device="cpu", dist=dist),
                DL.dml_plr_lasso(y, w, x, device="cpu", dist=dist)]

    for out in _run(fn, world, n):
        for a, b in zip(out, single):
            assert a.ate == pytest.approx(b.ate, rel=1e-7, abs=1e-10), a.method
            if np.isfinite(b.se):
                assert a.se == pytest.approx(b.se, rel=1e-7), a.method


@pytest.mark.parametrize("world", [2, 3])
def test_tree_parallel_forests_equal_single(world):
    """Trees sharded over ranks (C05): identical trees per global tree id; the OOB votes,
    the nuisance predictions and the causal-forest tau / variance are the SAME BITS as the
    single-device forest (int64 fixed-point prediction sums)."""
    from ate_replication_causalml_amd.models import forest as F
    r = np.random.default_rng(0)
    n = 1500
    X = r.normal(size=(n, 5))
    W = (r.uniform(size=n) < 0.4).astype(float)
    Y = X[:, 0] + (1 + (X[:, 1] > 0)) * W + 0.3 * r.normal(size=n)
    rf1 = F.rf_classifier(X, W, num_trees=24, seed=5, backend="cpu").oob_proba()
    cf1 = F.causal_forest(X, Y, W, num_trees=24, nuisance_trees=12, seed=9, backend="cpu")

    def fn(dist):
        fr = F.fit_forest_sharded(X, F.KIND_CLASS, 24, dist.comm, y=W, seed=5, backend="cpu")
        p = F.predict_tree_parallel(fr, dist.comm, oob=True)
        cf = F.causal_forest(X, Y, W, num_trees=24, nuisance_trees=12, seed=9, backend="cpu",
                             comm=dist.comm)
        return p, cf

    for p, cf in _run(fn, world, n):
        np.testing.assert_array_equal(p, rf1)
        np.testing.assert_array_equal(cf.y_hat, cf1.y_hat)
        np.testing.assert_array_equal(cf.w_hat, cf1.w_hat)
        np.testing.assert_array_equal(cf.tau_oob, cf1.tau_oob)
        np.testing.assert_array_equal(cf.var_oob, cf1.var_oob)


@pytest.mark.parametrize("world", [1, 3])
def test_reduce_scatter_and_all_gather_into(world):
    """Communicator primitives of the feature-sliced C04: reduce_scatter_ returns this rank's
    chunk of the rank-ordered sum, all_gather_into_ the rank-ordered concatenation."""
    from ate_replication_causalml_amd.parallel.comm import LocalComm

    def fn(comm):
        r = comm.rank
        t = torch.arange(4 * comm.world_size, dtype=torch.int64) * (r + 1)
        out = torch.empty(4, dtype=torch.int64)
        comm.reduce_scatter_(out, t)
        g = torch.empty(3 * comm.world_size, dtype=torch.int64)
        comm.all_gather_into_(g, torch.full((3,), r, dtype=torch.int64))
        return out, g

    res = [fn(LocalComm())] if world == 1 else run_simulated(world, fn)
    scale = sum(r + 1 for r in range(world))
    for r, (out, g) in enumerate(res):
        assert out.tolist() == [scale * v for v in range(4 * r, 4 * r + 4)]
        assert g.tolist() == [q for q in range(world) for _ in range(3)]
