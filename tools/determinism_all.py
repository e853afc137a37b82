"""Run-to-run determinism of every device estimator on one GPU: each runs three times
eagerly (graph=False where the estimator has a graph path) on identical data; prints
whether ATE and SE are bit-identical across the runs."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ate_replication_causalml_amd  # noqa: E402,F401
import numpy as np  # noqa: E402
import torch  # noqa: E402

from ate_replication_causalml_amd.estimators import balance, forest, lasso, linear  # noqa: E402

dev = torch.device("cuda", 0)
rs = np.random.RandomState(2)
n, p = 4000, 10
X = rs.randn(n, p)
W = (rs.rand(n) < 1 / (1 + np.exp(-0.7 * X[:, 0]))).astype(float)
Yc = X[:, 1] + 0.4 * W + rs.randn(n)
Yb = (rs.rand(n) < 1 / (1 + np.exp(-(X[:, 1] + 0.5 * W)))).astype(float)
ps = 1 / (1 + np.exp(-0.7 * X[:, 0]))
cases = {
    "ols": lambda: linear.ols(Yc, W, X, device=dev, graph=False),
    "ipw": lambda: linear.ipw(Yc, W, X, ps, device=dev, graph=False),
    "ipw_wls": lambda: linear.ipw_wls(Yc, W, ps, device=dev, graph=False),
    "aipw_glm": lambda: linear.aipw_glm(Yb, W, X, device=dev, graph=False),
    "aipw_glm_boot": lambda: linear.aipw_glm(Yb, W, X, bootstrap_se=True, B=200, device=dev,
                                             graph=False),
    "lasso_single": lambda: lasso.lasso_single(Yc, W, X, device=dev, graph=False),
    "belloni": lambda: lasso.belloni(Yc, W, X[:, :6], device=dev, graph=False),
    "dml": lambda: lasso.dml_plr_lasso(Yc, W, X, device=dev, graph=False),
    "aipw_rf": lambda: forest.aipw_rf(Yb, W, X, num_trees=80, device=dev, graph=False),
    "double_ml": lambda: forest.double_ml(Yb, W, X, num_trees=60, device=dev, graph=False),
    "causal_forest": lambda: forest.causal_forest_ate(Yc, W, X, num_trees=200, device=dev,
                                                      graph=False),
    "residual_balance": lambda: balance.residual_balance(Yc, W, X, device=dev),
}
bad = 0
for name, fn in cases.items():
    rs_ = [fn() for _ in range(3)]
    vals = {repr((r.ate, r.se)) for r in rs_}          # repr: NaN SE (LASSO rows) compares equal
    ok = len(vals) == 1
    bad += not ok
    print(f"{name:18s} {'bit-identical' if ok else 'DIFFERS'} ate={rs_[0].ate!r} "
          f"spread={max(r.ate for r in rs_) - min(r.ate for r in rs_):.2e}", flush=True)
print("all bit-identical" if not bad else f"{bad} estimator(s) differ run to run")
