"""Every device estimator is bit-reproducible run to run on one GPU (three eager runs on
identical data). Guards against races such as the two-writer slab reduce that made the
row-weighted Gram -- and through the interior point the residual-balancing ATE -- differ
at rounding level (tools/determinism_all.py runs the full sweep)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _data():
    rs = np.random.RandomState(2)
    n, p = 2500, 8
    X = rs.randn(n, p)
    W = (rs.rand(n) < 1 / (1 + np.exp(-0.7 * X[:, 0]))).astype(float)
    Yc = X[:, 1] + 0.4 * W + rs.randn(n)
    Yb = (rs.rand(n) < 1 / (1 + np.exp(-(X[:, 1] + 0.5 * W)))).astype(float)
    return X, W, Yc, Yb


def _cases(dev):
    from ate_replication_causalml_amd.estimators import balance, forest, lasso, linear
    X, W, Yc, Yb = _data()
    return {
        "ols": lambda: linear.ols(Yc, W, X, device=dev, graph=False),
        "aipw_glm": lambda: linear.aipw_glm(Yb, W, X, device=dev, graph=False),
        "lasso_single": lambda: lasso.lasso_single(Yc, W, X, device=dev, graph=False),
        "dml": lambda: lasso.dml_plr_lasso(Yc, W, X, device=dev, graph=False),
        "aipw_rf": lambda: forest.aipw_rf(Yb, W, X, num_trees=40, device=dev, graph=False),
        "causal_forest": lambda: forest.causal_forest_ate(Yc, W, X, num_trees=100, device=dev,
                                                          graph=False, compat="textbook"),
        # the production default: grf's AIPW without clipping W.hat (here in [0.15, 0.80])
        "causal_forest_reference": lambda: forest.causal_forest_ate(Yc, W, X, num_trees=100,
                                                                    device=dev, graph=False),
        "residual_balance": lambda: balance.residual_balance(Yc, W, X, device=dev),
    }


@pytest.mark.parametrize("name", ["ols", "aipw_glm", "lasso_single", "dml", "aipw_rf",
                                  "causal_forest", "causal_forest_reference",
                                  "residual_balance"])
def test_estimator_bit_reproducible(gpu, name):
    fn = _cases(gpu)[name]
    vals = {repr((r.ate, r.se)) for r in (fn() for _ in range(3))}
    assert len(vals) == 1, (name, vals)
