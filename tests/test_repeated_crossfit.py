"""Repeated cross-fitting for the K-fold DML (Chernozhukov et al. 2018 §3.4): S distinct
K-fold partitions from K*K micro-segments, one Gram pass shared by all partitions
(estimators/lasso.dml_repeated_phases), median aggregation -- against the float64 T-ref
(reference/estimators.dml_plr_lasso_repeated), across a simulated row sharding, and
through the public API. Reference ancestor: the 2-way split-and-average DML of
/root/reference/ate_functions.R:372-389."""
import itertools

import numpy as np
import pytest
import torch

import ate_replication_causalml_amd as ate
from ate_replication_causalml_amd.config import RunConfig
from ate_replication_causalml_amd.estimators import lasso as L
from ate_replication_causalml_amd.parallel.comm import LocalComm, run_simulated
from ate_replication_causalml_amd.reference import estimators as R


def _data(n=2500, p=10, seed=3):
    rs = np.random.RandomState(seed)
    X = rs.randn(n, p)
    W = (rs.rand(n) < 1 / (1 + np.exp(-X[:, 0]))).astype(float)
    Y = X[:, 1] + 0.5 * W + rs.randn(n)
    return Y, W, X


@pytest.mark.parametrize("K", [3, 5])
def test_micro_fold_partitions(K):
    """Every partition puts K micro-segments in each fold; for prime K all K partitions are
    distinct, and two of them share exactly one micro-segment per pair of folds."""
    maps = [L.micro_fold_map(K, s) for s in range(K)]
    for m in maps:
        assert np.array_equal(np.bincount(m, minlength=K), np.full(K, K))
    for s, t in itertools.combinations(range(K), 2):
        assert not np.array_equal(maps[s], maps[t])
        for i, j in itertools.product(range(K), repeat=2):
            assert np.sum((maps[s] == i) & (maps[t] == j)) == 1


def test_median_aggregate():
    th = torch.tensor([0.3, 0.1, 0.2, 0.5], dtype=torch.float64)
    se = torch.tensor([0.01, 0.02, 0.03, 0.04], dtype=torch.float64)
    t, s = L.median_aggregate(th, se).tolist()
    assert t == pytest.approx(0.25)
    assert s == pytest.approx(np.sqrt(np.median(se.numpy() ** 2 + (th.numpy() - 0.25) ** 2)))
    t3, _ = L.median_aggregate(th[:3], se[:3]).tolist()
    assert t3 == pytest.approx(0.2)
    tm, sm = L.median_aggregate(th, se, "mean").tolist()
    assert tm == pytest.approx(th.mean().item())
    assert sm == pytest.approx(np.sqrt(np.mean(se.numpy() ** 2 + (th.numpy() - tm) ** 2)))


@pytest.mark.parametrize("repeats,aggregate", [(3, "median"), (4, "median"), (2, "mean")])
def test_repeated_dml_matches_tref(repeats, aggregate):
    """The device pipeline on host tensors (one K*K micro-Gram stack, per-partition fold
    Grams, CV-LASSO paths, residual moments, aggregate) equals the T-ref, which refits each
    partition from scratch with glmnet-equivalent CV on row subsets."""
    Y, W, X = _data()
    a = R.dml_plr_lasso_repeated(Y, W, X, 5, repeats, aggregate=aggregate)
    b = L.dml_plr_lasso_repeated(Y, W, X, 5, repeats, aggregate=aggregate, device="cpu")
    np.testing.assert_allclose(np.array(b.diagnostics["splits"]),
                               np.array(a.diagnostics["splits"]), rtol=1e-9)
    assert b.ate == pytest.approx(a.ate, rel=1e-9) and b.se == pytest.approx(a.se, rel=1e-9)
    th = np.array(a.diagnostics["splits"])[:, 0]
    assert len(set(np.round(th, 12))) == repeats          # distinct partitions, distinct fits


def test_repeated_one_partition_is_a_dml_fit():
    """S = 1 is one K-fold DML over the folds a = micro // K."""
    from ate_replication_causalml_amd.parallel import rng
    Y, W, X = _data(1500, 8, 5)
    micro = rng.fold_ids(len(Y), 25, 1991, 0)
    one = R.dml_plr_lasso(Y, W, X, 5, fold_ids=micro // 5)
    r = L.dml_plr_lasso_repeated(Y, W, X, 5, 1, device="cpu")
    assert r.ate == pytest.approx(one.ate, rel=1e-9) and r.se == pytest.approx(one.se, rel=1e-9)


def test_repeated_dml_row_sharded():
    """Row shards (thread simulator, world 3): the micro-Gram stack and the per-partition
    moments are all-reduced; the same aggregate as world 1."""
    from ate_replication_causalml_amd.data.device_dgp import synthetic_panel

    def run(world, rank, comm):
        pan = synthetic_panel(3000, p=24, folds=25, seed=3, dtype="f64", device="cpu",
                              rank=rank, world=world)
        res, splits = L.dml_repeated_panel(pan, 5, 3, comm=comm)
        return res.numpy(), splits.numpy()
    ref, rsp = run(1, 0, LocalComm())
    for res, sp in run_simulated(3, lambda c: run(3, c.rank, c)):
        np.testing.assert_allclose(res, ref, rtol=1e-9)
        np.testing.assert_allclose(sp, rsp, rtol=1e-9)


def test_api_repeats():
    Y, W, X = _data(1500, 8, 7)
    a = ate.ate_dml(Y, W, X, repeats=3, run=RunConfig(backend="reference"))
    b = ate.ate_dml(Y, W, X, repeats=3, run=RunConfig(backend="cpu"))
    assert b.ate == pytest.approx(a.ate, rel=1e-9) and b.diagnostics["repeats"] == 3
