"""Approximate residual balancing (E14): the IPM QP solver against an independent
SLSQP solve, and the device orchestration (CPU tensors) against the float64 T-ref."""
import numpy as np
import pytest
from scipy.optimize import minimize

from ate_replication_causalml_amd.reference import balance as B


@pytest.mark.parametrize("n,p", [(40, 3), (120, 6)])
def test_ipm_matches_slsqp(n, p):
    r = np.random.default_rng(n)
    M = r.normal(size=(n, p)) + 0.3
    m = M.mean(0) + 0.2
    g, info = B.ipm_balance(M, m)
    assert abs(g.sum() - 1) < 1e-9 and g.min() > -1e-12

    def f(v):
        return 0.5 * v[:n] @ v[:n] + 0.5 * v[n] ** 2

    cons = [{"type": "eq", "fun": lambda v: v[:n].sum() - 1},
            {"type": "ineq", "fun": lambda v: v[n] - (M.T @ v[:n] - m)},
            {"type": "ineq", "fun": lambda v: v[n] + (M.T @ v[:n] - m)}]
    res = minimize(f, np.r_[np.full(n, 1 / n), 1.0], constraints=cons,
                   bounds=[(0, None)] * n + [(None, None)], method="SLSQP",
                   options={"ftol": 1e-14, "maxiter": 2000})
    assert info["objective"] <= B.balance_objective(M, m, res.x[:n]) + 1e-10
    assert np.abs(g - res.x[:n]).max() < 1e-5


def test_ipm_negative_weights_closed_form():
    # without gamma >= 0 and with zeta -> objective is smooth on the active set; check KKT:
    r = np.random.default_rng(3)
    M = r.normal(size=(60, 4))
    m = np.zeros(4)
    g, info = B.ipm_balance(M, m, allow_negative=True)
    assert abs(g.sum() - 1) < 1e-9
    assert info["objective"] <= B.balance_objective(M, m, np.full(60, 1 / 60)) + 1e-12


def test_scale_columns_keeps_binary():
    X = np.column_stack([np.r_[0, 1, 1, 0], np.r_[1.0, 2.0, 3.0, 4.0]])
    Xs, scl = B.scale_columns(X)
    assert scl[0] == 1.0 and scl[1] == pytest.approx(np.std([1, 2, 3, 4], ddof=1))


def test_device_arb_matches_reference(tutorial):
    from ate_replication_causalml_amd.estimators.balance import residual_balance
    _, m, _ = tutorial
    a = B.residual_balance_ate(m.Y, m.W, m.X)
    b = residual_balance(m.Y, m.W, m.X, device="cpu")
    assert b.ate == pytest.approx(a.ate, abs=1e-9)
    assert b.se == pytest.approx(a.se, rel=1e-7)


def test_fixed_budget_ipm_equals_early_stop():
    """The capturable interior point (fixed iteration budget, converged arms frozen with
    torch.where, device iteration counts) returns exactly the early-stopping solver's
    weights and iteration counts (host tensors)."""
    import numpy as np
    import torch
    from ate_replication_causalml_amd.estimators import balance as B
    from ate_replication_causalml_amd.ops.panel import build_panel
    from ate_replication_causalml_amd.parallel import rng
    from ate_replication_causalml_amd.reference.balance import scale_columns
    rs = np.random.RandomState(3)
    n, p, K = 1200, 6, 5
    X = rs.randn(n, p)
    W = (rs.rand(n) < 0.35).astype(float)
    Y = X[:, 1] + 0.4 * W + rs.randn(n)
    Xs = scale_columns(X)[0]
    arm = W == 1
    seg = np.empty(n, dtype=np.int64)
    seg[arm] = rng.fold_ids(int(arm.sum()), K, 1991, 10)
    seg[~arm] = K + rng.fold_ids(int((~arm).sum()), K, 1991, 11)
    pan = build_panel(Xs, None, Y, folds=seg, dtype="f64", device="cpu")
    masks = B._arm_masks(pan, K)
    tg = torch.as_tensor(Xs.mean(0))
    g1, i1 = B.ipm_balance_panel(pan, masks, tg, 0.5)
    nr = np.asarray(pan.seg_nreal)
    sa = tuple(int(s // K) if nr[s] > 0 else -1 for s in range(pan.nseg))
    g2, i2 = B.ipm_balance_panel(pan, masks, tg, 0.5, seg_arm=sa, fixed=True)
    assert torch.equal(g1, g2)
    assert list(i1) == i2.tolist()


@pytest.mark.parametrize("fixed", [False, True])
def test_converged_arm_nan_solve_does_not_leak(fixed, monkeypatch):
    """A converged arm whose Schur system loses its positive pivots (spd_solve -> NaN) must
    not poison the arm still iterating: its solution is zeroed before the mask products
    (ADVICE r02). NaN is injected into arm 0's solve from the iteration it converged at."""
    import torch
    from ate_replication_causalml_amd.estimators import balance as EB
    from ate_replication_causalml_amd.ops.panel import build_panel
    from ate_replication_causalml_amd.parallel import rng
    rs = np.random.RandomState(5)
    n, p, K = 900, 5, 5
    X = rs.randn(n, p)
    W = (rs.rand(n) < 0.3).astype(float)
    Y = X[:, 0] + 0.5 * W + rs.randn(n)
    Xs = B.scale_columns(X)[0]
    arm = W == 1
    seg = np.empty(n, dtype=np.int64)
    seg[arm] = rng.fold_ids(int(arm.sum()), K, 1991, 10)
    seg[~arm] = K + rng.fold_ids(int((~arm).sum()), K, 1991, 11)
    pan = build_panel(Xs, None, Y, folds=seg, dtype="f64", device="cpu")
    masks = EB._arm_masks(pan, K)
    tg = torch.as_tensor(Xs.mean(0))
    nr = np.asarray(pan.seg_nreal)
    sa = tuple(int(s // K) if nr[s] > 0 else -1 for s in range(pan.nseg))
    g_ref, it_ref = EB.ipm_balance_panel(pan, masks, tg, 0.5, seg_arm=sa, fixed=fixed)
    it_ref = [int(v) for v in (it_ref.tolist() if fixed else it_ref)]
    first = int(np.argmin(it_ref))
    assert it_ref[first] < it_ref[1 - first], "arms must converge at different iterations"
    real = EB.spd_solve
    calls = {"n": 0}

    def poisoned(Kmat, r):
        x = real(Kmat, r)
        calls["n"] += 1
        it = (calls["n"] + 1) // 2             # two solves per iteration
        if it > it_ref[first]:
            x = x.clone()
            x[first] = float("nan")
        return x
    monkeypatch.setattr(EB, "spd_solve", poisoned)
    g, it = EB.ipm_balance_panel(pan, masks, tg, 0.5, seg_arm=sa, fixed=fixed)
    assert torch.isfinite(g).all()
    assert torch.equal(g, g_ref)


def test_device_arb_allow_negative_matches_reference(tutorial):
    """allow.negative.weights runs the device interior point without the gamma >= 0
    barrier (no silent host fallback) and matches the T-ref."""
    from ate_replication_causalml_amd.estimators.balance import residual_balance
    _, m, _ = tutorial
    a = B.residual_balance_ate(m.Y, m.W, m.X, allow_negative=True)
    b = residual_balance(m.Y, m.W, m.X, device="cpu", allow_negative=True)
    assert b.ate == pytest.approx(a.ate, abs=1e-8)
    assert b.se == pytest.approx(a.se, rel=1e-6)
    c = residual_balance(m.Y, m.W, m.X, device="cpu")
    assert abs(c.ate - b.ate) > 1e-9          # the constraint matters on this data
