"""Cross-fitted AIPW (config 3) and causal-forest bootstrap SE (config 4)."""
import numpy as np
import pytest

from ate_replication_causalml_amd.estimators import crossfit as CF
from ate_replication_causalml_amd.models import forest as F
from ate_replication_causalml_amd.parallel.comm import run_simulated


def _toy(n=3000, seed=0):
    r = np.random.default_rng(seed)
    X = r.normal(size=(n, 6))
    e = 1 / (1 + np.exp(-(0.5 * X[:, 0] - 0.3 * X[:, 1])))
    W = (r.uniform(size=n) < e).astype(float)
    p0 = 1 / (1 + np.exp(-(X[:, 0] + 0.5 * X[:, 2])))
    p1 = 1 / (1 + np.exp(-(X[:, 0] + 0.5 * X[:, 2] + 0.8)))
    Y = (r.uniform(size=n) < np.where(W == 1, p1, p0)).astype(float)
    return X, W, Y, float((p1 - p0).mean())


@pytest.mark.parametrize("learner", ["glm", "rf"])
def test_aipw_crossfit_recovers_effect(learner):
    X, W, Y, tau = _toy()
    r = CF.aipw_crossfit(Y, W, X, learner=learner, num_trees=60, device="cpu")
    assert abs(r.ate - tau) < 4 * r.se + 0.01
    assert 0.005 < r.se < 0.1


def test_aipw_crossfit_glm_matches_manual():
    """glm learner == hand-rolled cross-fit with the reference logistic regression."""
    from ate_replication_causalml_amd.parallel import rng
    from ate_replication_causalml_amd.reference.linear import glm_logit, glm_predict
    X, W, Y, _ = _toy(1500, 1)
    n = len(Y)
    fid = rng.fold_ids(n, 5, 1991, 11)
    e, m1, m0 = np.empty(n), np.empty(n), np.empty(n)
    for k in range(5):
        ho, tr = fid == k, fid != k
        e[ho] = glm_predict(glm_logit(X[tr], W[tr]), X[ho])
        t1, t0 = tr & (W == 1), tr & (W == 0)
        m1[ho] = glm_predict(glm_logit(X[t1], Y[t1]), X[ho])
        m0[ho] = glm_predict(glm_logit(X[t0], Y[t0]), X[ho])
    e = np.clip(e, 0.01, 0.99)
    g = m1 - m0 + W * (Y - m1) / e - (1 - W) * (Y - m0) / (1 - e)
    r = CF.aipw_crossfit(Y, W, X, learner="glm", device="cpu")
    assert r.ate == pytest.approx(g.mean(), rel=1e-8)
    assert r.se == pytest.approx(g.std(ddof=1) / np.sqrt(n), rel=1e-8)


def test_crossfit_and_cf_bootstrap_tree_parallel():
    X, W, Y, _ = _toy(1200, 2)
    a1 = CF.aipw_crossfit(Y, W, X, learner="rf", num_trees=16, device="cpu")
    b1 = CF.causal_forest_bootstrap(Y, W, X, num_trees=24, nuisance_trees=12, B=50, compat="textbook", device="cpu")

    def fn(comm):
        return (CF.aipw_crossfit(Y, W, X, learner="rf", num_trees=16, device="cpu", comm=comm),
                CF.causal_forest_bootstrap(Y, W, X, num_trees=24, nuisance_trees=12, B=50, compat="textbook",
                                           device="cpu", comm=comm))

    for a, b in run_simulated(2, fn):          # fixed-point forest sums: the same bits
        assert a.ate == a1.ate and a.se == a1.se
        assert b.ate == b1.ate and b.se == b1.se


class _Killed(RuntimeError):
    pass


@pytest.mark.parametrize("learner", ["rf", "glm"])
def test_aipw_crossfit_checkpoint_resume(learner, tmp_path, monkeypatch):
    """A cross-fit killed after fold 2 resumes from its per-(fold, nuisance) checkpoints:
    only the missing nuisances are refit and the ATE / SE are bitwise identical."""
    from ate_replication_causalml_amd.utils.checkpoint import Checkpoint
    X, W, Y, _ = _toy(1500, 4)
    kw = dict(learner=learner, num_trees=12, device="cpu")
    want = CF.aipw_crossfit(Y, W, X, **kw)
    name = "_rf_fit_predict" if learner == "rf" else "_glm_fit_predict"
    real = getattr(CF, name)
    calls = {"n": 0, "die": 9}                  # folds 0-2 = 9 nuisance fits

    def counted(*a, **k):
        calls["n"] += 1
        if calls["n"] > calls["die"]:
            raise _Killed()
        return real(*a, **k)
    monkeypatch.setattr(CF, name, counted)
    ck = Checkpoint(tmp_path, {"cfg": "aipw"})
    with pytest.raises(_Killed):
        CF.aipw_crossfit(Y, W, X, checkpoint=ck, **kw)
    assert len(list(tmp_path.glob("aipw_fold*.npz"))) == 9
    calls.update(n=0, die=10 ** 9)
    got = CF.aipw_crossfit(Y, W, X, checkpoint=ck, **kw)
    assert calls["n"] == 6                      # folds 3 and 4 only
    assert got.ate == want.ate and got.se == want.se


def test_cf_bootstrap_checkpoint_resume(tmp_path, monkeypatch):
    """Config 4: the forest outputs and the bootstrap ranges are checkpointed; a run
    killed after the first replicate range resumes to the identical SE."""
    from ate_replication_causalml_amd.estimators import linear as L
    from ate_replication_causalml_amd.utils.checkpoint import Checkpoint
    X, W, Y, _ = _toy(800, 5)
    kw = dict(num_trees=16, nuisance_trees=8, B=60, device="cpu", boot_chunk=20, compat="textbook")
    want = CF.causal_forest_bootstrap(Y, W, X, **kw)
    real = L.bootstrap_replicates
    calls = {"n": 0, "die": 1}

    def counted(*a, **k):
        calls["n"] += 1
        if calls["n"] > calls["die"]:
            raise _Killed()
        return real(*a, **k)
    monkeypatch.setattr(L, "bootstrap_replicates", counted)
    ck = Checkpoint(tmp_path, {"cfg": 4})
    with pytest.raises(_Killed):
        CF.causal_forest_bootstrap(Y, W, X, checkpoint=ck, **kw)
    calls.update(n=0, die=10 ** 9)
    from ate_replication_causalml_amd.models import forest as F
    monkeypatch.setattr(F, "causal_forest", lambda *a, **k: (_ for _ in ()).throw(
        AssertionError("the forest must come from the checkpoint")))
    got = CF.causal_forest_bootstrap(Y, W, X, checkpoint=ck, **kw)
    assert calls["n"] == 2                       # replicate ranges 2 and 3 only
    assert got.ate == want.ate and got.se == want.se


def test_cf_bootstrap_resume_ranks_agree(tmp_path):
    """Two simulated ranks resume a config-4 run in which ONE rank lost its forest and one
    of its bootstrap ranges (a kill between the ranks' saves): every rank must recompute
    the same stages (the tree-sharded forest and the all-gathered replicates pair up
    across ranks), so the run completes and equals the uninterrupted one bit for bit."""
    from ate_replication_causalml_amd.utils.checkpoint import Checkpoint
    X, W, Y, _ = _toy(600, 6)
    kw = dict(num_trees=16, nuisance_trees=8, B=40, device="cpu", boot_chunk=20, compat="textbook")

    def fn(comm):
        ck = Checkpoint(tmp_path, {"cfg": 4})
        return CF.causal_forest_bootstrap(Y, W, X, checkpoint=ck, comm=comm, **kw)

    want = run_simulated(2, fn)
    gone = [*tmp_path.glob("cf_fit.r1of2.*.npz"), *tmp_path.glob("cf_boot_20_40.r1of2.*.npz")]
    assert len(gone) == 2
    for f in gone:
        f.unlink()
    got = run_simulated(2, fn)
    for a, b in zip(got, want):
        assert a.ate == b.ate and a.se == b.se


def test_rf_panel_crossfit_tree_parallel_bitwise():
    """Config 3 on a panel (host twin of the HBM path): the forests' local held-out vote
    sums are packed and all-reduced ONCE (C05); votes are integers, so 2 and 3 ranks give
    the SAME BITS as one process; a 1/2 tree shard alone differs (it has half the trees)."""
    from ate_replication_causalml_amd.data.device_dgp import synthetic_panel
    pan = synthetic_panel(3000, p=24, folds=5, seed=5, dtype="f32", device="cpu")
    one = CF.aipw_rf_crossfit_panel(pan, num_trees=12, seed=3)
    assert np.isfinite(one.ate) and one.se > 0
    for world in (2, 3):
        for r in run_simulated(world, lambda c: CF.aipw_rf_crossfit_panel(
                pan, num_trees=12, seed=3, comm=c)):
            assert r.ate == one.ate and r.se == one.se
            assert r.diagnostics["trees_this_device"] in (12 // world, 12 // world + 1)
    half = CF.aipw_rf_crossfit_panel(pan, num_trees=12, seed=3, tree_shard=(0, 2))
    assert half.ate != one.ate


def test_rf_panel_crossfit_checkpoint_resume_two_ranks(tmp_path, monkeypatch):
    """Killed after some forests on one rank, the config-3 panel cross-fit resumes from the
    per-rank local vote sums: every rank agrees which jobs to regrow, and the resumed ATE/SE
    equal the uninterrupted run's bits."""
    from ate_replication_causalml_amd.data.device_dgp import synthetic_panel
    from ate_replication_causalml_amd.utils.checkpoint import Checkpoint
    pan = synthetic_panel(2000, p=21, folds=5, seed=9, dtype="f32", device="cpu")
    want = CF.aipw_rf_crossfit_panel(pan, num_trees=8, seed=2)

    def fn(c):
        return CF.aipw_rf_crossfit_panel(pan, num_trees=8, seed=2, comm=c,
                                         checkpoint=Checkpoint(tmp_path, {"cfg": 3}),
                                         data_key="syn")
    run_simulated(2, fn)
    files = sorted(tmp_path.glob("aipw_fold*.r1of2.*.npz"))
    assert len(files) == 15
    for f in files[:4]:
        f.unlink()                        # rank 1 lost 4 jobs; rank 0 still has them
    real = F.fit_forest_binned
    calls = {"n": 0}

    def counted(*a, **k):
        calls["n"] += 1
        return real(*a, **k)
    monkeypatch.setattr(F, "fit_forest_binned", counted)
    got = run_simulated(2, fn)
    assert calls["n"] == 8                # the 4 lost jobs, regrown on both ranks
    for r in got:
        assert r.ate == want.ate and r.se == want.se
