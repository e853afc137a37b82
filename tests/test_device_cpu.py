"""The device-path orchestration (estimators/ + ops/) executed with CPU tensors
(float64 torch implementations of every op) must reproduce the float64 reference
exactly; on the GPU the same orchestration runs the HIP kernels (tests/test_gpu.py)."""
import numpy as np
import pytest
import torch

from ate_replication_causalml_amd.estimators import lasso as DL
from ate_replication_causalml_amd.estimators import linear as D
from ate_replication_causalml_amd.ops import gram as gram_op
from ate_replication_causalml_amd.ops.linalg import chol_solve
from ate_replication_causalml_amd.ops.panel import build_panel
from ate_replication_causalml_amd.reference import estimators as E

CPU = torch.device("cpu")


def close(a, b, tol=1e-9):
    assert a.ate == pytest.approx(b.ate, abs=tol, rel=tol)
    if not np.isnan(a.se):
        assert a.se == pytest.approx(b.se, abs=tol, rel=tol)


def test_panel_layout_fold_contiguous():
    rs = np.random.RandomState(0)
    X = rs.randn(130, 3)
    folds = rs.randint(0, 3, 130)
    pan = build_panel(X, rs.rand(130), rs.rand(130), folds=folds, dtype="f64", device=CPU)
    assert pan.ld % 64 == 0 and pan.P % 64 == 0
    for k, (r0, r1) in enumerate(pan.seg_bounds):
        assert (r1 - r0) % 64 == 0
        idx = pan.row_index[r0:r1]
        real = idx[idx >= 0].numpy()
        assert (folds[real] == k).all()
        assert pan.valid()[r0:r1].sum() == (folds == k).sum()
    back = pan.scatter_rows(pan.col("x1"))
    assert np.allclose(back.numpy(), X[:, 1])


@pytest.mark.parametrize("dtype", ["f64", "f32", "bf16"])
def test_panel_from_tensor_equals_host_build(dtype):
    rs = np.random.RandomState(1)
    X = rs.randn(300, 7)
    folds = rs.randint(0, 4, 300)
    w, y = rs.rand(300), rs.rand(300)
    a = build_panel(X, w, y, folds=folds, dtype=dtype, device=CPU, extra_cols=("s",))
    b = build_panel(torch.from_numpy(X), w, y, folds=folds, dtype=dtype, device=CPU,
                    extra_cols=("s",))
    assert a.cols == b.cols and a.xcols == b.xcols
    assert torch.equal(a.data, b.data)
    assert torch.equal(a.row_index, b.row_index)


def test_gram_cpu_matches_numpy():
    rs = np.random.RandomState(1)
    X = rs.randn(200, 5)
    pan = build_panel(X, rs.rand(200), rs.rand(200), folds=rs.randint(0, 2, 200), device=CPU)
    G = gram_op.gram(pan)
    A = pan.data.double().numpy()
    ref = sum(A[:, r0:r1] @ A[:, r0:r1].T for r0, r1 in pan.seg_bounds)
    assert np.allclose(G.sum(0).numpy(), ref)


def test_chol_solve_aliasing_cpu():
    rs = np.random.RandomState(2)
    X = rs.randn(300, 4)
    X[:, 3] = X[:, 1] + X[:, 2]
    y = rs.randn(300)
    pan = build_panel(X, None, y, device=CPU)
    G = gram_op.gram(pan)[0]
    cols = [pan.cols["one"], *pan.xcols]
    r = chol_solve(G, cols, pan.cols["Y"])
    from ate_replication_causalml_amd.reference.linear import lm_fit
    f = lm_fit(X, y)
    assert np.array_equal(np.isnan(r.beta.numpy()), f.aliased)
    assert np.allclose(np.nan_to_num(r.beta.numpy()), np.nan_to_num(f.coef))


def test_linear_family_matches_reference(tutorial):
    _, m, _ = tutorial
    Y, W, X = m.Y, m.W, m.X
    close(D.naive(Y, W, device=CPU), E.naive(Y, W))
    close(D.ols(Y, W, X, device=CPU), E.ols(Y, W, X))
    p = E.propensity_logistic(W, X)
    pd = D.propensity_logistic(W, X, device=CPU).numpy()
    assert np.abs(p - pd).max() < 1e-10
    for compat in ("reference", "textbook"):
        close(D.ipw(Y, W, X, p, compat=compat, device=CPU), E.ipw(Y, W, X, p, compat=compat))
    close(D.ipw_wls(Y, W, p, device=CPU), E.ipw_wls(Y, W, p))
    close(D.aipw_glm(Y, W, X, device=CPU), E.aipw_glm(Y, W, X), tol=1e-8)
    close(D.aipw_glm(Y, W, X, bootstrap_se=True, B=20, device=CPU),
          E.aipw_glm(Y, W, X, bootstrap_se=True, B=20), tol=1e-8)


def test_lasso_family_matches_reference(tutorial):
    _, m, _ = tutorial
    Y, W, X = m.Y, m.W, m.X
    close(DL.lasso_single(Y, W, X, device=CPU), E.lasso_single(Y, W, X), tol=1e-7)
    close(DL.lasso_usual(Y, W, X, device=CPU), E.lasso_usual(Y, W, X), tol=1e-7)
    close(DL.dml_plr_lasso(Y, W, X, device=CPU), E.dml_plr_lasso(Y, W, X), tol=1e-7)


@pytest.mark.slow
def test_belloni_matches_reference(tutorial):
    _, m, _ = tutorial
    Y, W, X = m.Y[:2500], m.W[:2500], m.X[:2500, :8]
    a, b = DL.belloni(Y, W, X, device=CPU), E.belloni(Y, W, X)
    close(a, b, tol=1e-7)
    assert a.diagnostics["n_selected"] == b.diagnostics["n_selected"]


def test_synthetic_panel_cpu_matches_host_dgp():
    from ate_replication_causalml_amd.data import dgp
    from ate_replication_causalml_amd.data.device_dgp import synthetic_panel
    pan = synthetic_panel(300, p=25, folds=3, seed=11, dtype="f64", device=CPU)
    cts, binc, extra, W, Y, _ = dgp.raw_columns(300, 11, 4)
    X = np.column_stack([cts, binc, extra])
    got = pan.scatter_rows(torch.stack([pan.col(f"x{j}") for j in range(25)], 1))
    assert np.allclose(got.numpy(), X)
    assert np.allclose(pan.scatter_rows(pan.col("W")).numpy(), W)


def test_propensity_lasso_device_orchestration(tutorial):
    from ate_replication_causalml_amd.estimators import linear as D
    from ate_replication_causalml_amd.reference import estimators as E
    _, m, _ = tutorial
    a = E.propensity_lasso(m.W, m.X)
    b = D.propensity_lasso(m.W, m.X, device="cpu").numpy()
    np.testing.assert_allclose(b, a, atol=1e-10)
