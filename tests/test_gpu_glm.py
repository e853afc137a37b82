"""GPU binomial CV-LASSO (csrc/lognet.hip) and device residual balancing vs the
float64 references."""
import numpy as np
import pytest
import torch

from ate_replication_causalml_amd.ops.lognet import cv_lognet
from ate_replication_causalml_amd.ops.panel import build_panel
from ate_replication_causalml_amd.parallel import rng
from ate_replication_causalml_amd.reference import glmnet as gn

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("p,alpha,dtype", [(12, 1.0, "f64"), (40, 0.7, "f64"), (12, 1.0, "f32")])
def test_lognet_cv_gpu_vs_reference(gpu, p, alpha, dtype):
    r = np.random.default_rng(p)
    n = 3000
    X = r.normal(size=(n, p))
    X[:, 0] = (X[:, 0] > 0)
    eta = -0.4 + X[:, :4] @ np.array([0.8, -0.5, 0.3, 0.2])
    y = (r.uniform(size=n) < 1 / (1 + np.exp(-eta))).astype(float)
    fid = rng.fold_ids(n, 10, 5, 3)
    pan = build_panel(X, None, y, folds=fid, dtype=dtype, device=gpu)
    cv = cv_lognet(pan, pan.xcols, pan.cols["Y"], alpha=alpha)
    Xr = pan.data.double().cpu()
    ref = gn.cv_glmnet(X if dtype == "f64" else X.astype(np.float32).astype(np.float64), y,
                       family="binomial", alpha=alpha, foldid=fid)
    m = int(cv.nlam[0])
    assert m == len(ref.lambdas)
    np.testing.assert_allclose(cv.lambdas[:m].cpu().numpy(), ref.lambdas, rtol=1e-9)
    np.testing.assert_allclose(cv.cvm[:m].cpu().numpy(), ref.cvm, rtol=1e-7)
    sel = cv.sel.cpu().numpy()
    assert (sel[0], sel[1]) == (ref.idx_min, ref.idx_1se)
    a0, b = ref.coef()
    np.testing.assert_allclose(cv.coef_1se.cpu().numpy(), np.r_[a0, b], atol=1e-7)


@pytest.mark.parametrize("p,dtype", [(12, "f64"), (40, "f32")])
def test_lognet_concurrent_equals_two_launch(gpu, p, dtype):
    """One-launch form (folds follow the full fit's lambdas through device flags) gives
    the same bits as the full-then-folds two-launch form."""
    r = np.random.default_rng(7 + p)
    n = 4000
    X = r.normal(size=(n, p))
    eta = 0.2 + X[:, :3] @ np.array([0.6, -0.4, 0.3])
    y = (r.uniform(size=n) < 1 / (1 + np.exp(-eta))).astype(float)
    pan = build_panel(X, None, y, folds=rng.fold_ids(n, 10, 5, 9), dtype=dtype, device=gpu)
    a = cv_lognet(pan, pan.xcols, pan.cols["Y"], concurrent=True)
    b = cv_lognet(pan, pan.xcols, pan.cols["Y"], concurrent=False)
    assert (a.npass.cpu().numpy() >= 0).all()
    assert torch.equal(a.nlam.cpu(), b.nlam.cpu())
    assert torch.equal(a.npass.cpu(), b.npass.cpu())
    m = int(a.nlam[0])
    for f in ("lambdas", "cvm", "cvsd"):
        assert torch.equal(getattr(a, f)[:m].cpu(), getattr(b, f)[:m].cpu()), f
    assert torch.equal(a.coef_path[:m].cpu(), b.coef_path[:m].cpu())
    assert torch.equal(a.sel.cpu(), b.sel.cpu())


def test_propensity_lasso_gpu(gpu, tutorial):
    from ate_replication_causalml_amd.estimators import linear as D
    from ate_replication_causalml_amd.reference import estimators as E
    _, m, _ = tutorial
    a = E.propensity_lasso(m.W, m.X)
    b = D.propensity_lasso(m.W, m.X, device=gpu).cpu().numpy()
    np.testing.assert_allclose(b, a, atol=1e-8)


def test_residual_balance_gpu(gpu, tutorial):
    from ate_replication_causalml_amd.estimators.balance import residual_balance
    from ate_replication_causalml_amd.reference.balance import residual_balance_ate
    _, m, _ = tutorial
    a = residual_balance_ate(m.Y, m.W, m.X)
    b = residual_balance(m.Y, m.W, m.X, device=gpu)
    assert b.ate == pytest.approx(a.ate, abs=1e-8)
    assert b.se == pytest.approx(a.se, rel=1e-6)


@pytest.mark.parametrize("dtype", ["f32", "f64"])
def test_panel_gemv_kernels(gpu, dtype):
    from ate_replication_causalml_amd.ops import gemv
    r = np.random.default_rng(1)
    n, p = 5000, 17
    X = r.normal(size=(n, p))
    pan = build_panel(X, None, r.normal(size=n), dtype=dtype, device=gpu)
    grp = torch.full((pan.ld,), -1, dtype=torch.int8, device=gpu)
    grp[: pan.n] = torch.as_tensor(r.integers(0, 2, pan.n), dtype=torch.int8, device=gpu)
    v = torch.as_tensor(r.normal(size=pan.ld), device=gpu)
    M = pan.data[pan.xcols].double().cpu()
    g = grp.cpu().long()
    ref = torch.stack([M @ torch.where(g == a, v.cpu(), torch.zeros_like(v.cpu())) for a in range(2)])
    out = gemv.xtv(pan, pan.xcols, v, grp, 2).cpu()
    torch.testing.assert_close(out, ref, rtol=1e-10, atol=1e-9)
    V = torch.as_tensor(r.normal(size=(2, p)), device=gpu)
    full = V.cpu() @ M
    ref2 = torch.where(g >= 0, full.gather(0, g.clamp(min=0)[None])[0], torch.zeros(pan.ld,
                                                                                     dtype=torch.float64))
    torch.testing.assert_close(gemv.xv(pan, pan.xcols, V, grp).cpu(), ref2, rtol=1e-10, atol=1e-9)


@pytest.mark.parametrize("compat", ["reference", "textbook"])
def test_device_selection_matches_host(gpu, compat):
    from ate_replication_causalml_amd.data.device_selection import keep_indices
    from ate_replication_causalml_amd.data.dgp import make_tutorial_data
    d = make_tutorial_data(n=50000, seed=1991)
    a = keep_indices(d.X, d.W, d.names, compat=compat, device=gpu).cpu().numpy()
    b = keep_indices(d.X, d.W, d.names, compat=compat, device="cpu").numpy()
    np.testing.assert_array_equal(a, b)
