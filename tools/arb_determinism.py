"""Run-to-run determinism of residual balancing (E14) on one GPU: the CV elastic net
coefficients and the interior-point weights, three eager runs on the same data."""
import hashlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ate_replication_causalml_amd  # noqa: E402,F401
import numpy as np  # noqa: E402
import torch  # noqa: E402

from ate_replication_causalml_amd.estimators import balance as B  # noqa: E402
from ate_replication_causalml_amd.ops.enet import cv_enet_gaussian  # noqa: E402
from ate_replication_causalml_amd.ops.gram import gram  # noqa: E402
from ate_replication_causalml_amd.ops.panel import build_panel  # noqa: E402
from ate_replication_causalml_amd.parallel import rng  # noqa: E402
from ate_replication_causalml_amd.reference.balance import scale_columns  # noqa: E402

dev = torch.device("cuda", 0)
rs = np.random.RandomState(11)
n, p, K = 3000, 8, 10
X = rs.randn(n, p)
W = np.zeros(n)
W[np.argsort(X[:, 0] + X[:, 2])[-1000:]] = 1
Y = X[:, 1] + 0.4 * W + rs.randn(n)
Xs = scale_columns(X)[0]
arm = W == 1
seg = np.empty(n, dtype=np.int64)
seg[arm] = rng.fold_ids(int(arm.sum()), K, 1991, 10)
seg[~arm] = K + rng.fold_ids(int((~arm).sum()), K, 1991, 11)
h = lambda t: hashlib.sha1(t.detach().cpu().numpy().tobytes()).hexdigest()[:12]  # noqa: E731
for rep in range(3):
    pan = build_panel(Xs, None, Y, folds=seg, dtype="f64", device=dev)
    G = gram(pan).clone()
    cv = cv_enet_gaussian(G, pan, pan.xcols, [pan.cols["Y"]],
                          full_sets=[list(range(K)), list(range(K, 2 * K))], alpha=0.9)
    masks = B._arm_masks(pan, K)
    gam, it = B.ipm_balance_panel(pan, masks, torch.as_tensor(Xs.mean(0)), 0.5)
    r = B.residual_balance(Y, W, X, device=dev)
    print(rep, "G", h(G), "cv", h(cv.coef_1se), "gam", h(gam), it, f"ate {r.ate:.17g}", flush=True)

# pieces of one IPM step, three times each on identical inputs
from ate_replication_causalml_amd.ops import gemv  # noqa: E402
from ate_replication_causalml_amd.ops.linalg import spd_solve  # noqa: E402
pan = build_panel(Xs, None, Y, folds=seg, dtype="f64", device=dev)
masks = B._arm_masks(pan, K)
grp = torch.where(masks[0], 0, torch.where(masks[1], 1, -1)).to(torch.int8)
g = torch.Generator().manual_seed(1)
v = torch.rand(pan.ld, generator=g, dtype=torch.float64).to(dev)
V = torch.rand(2, p, generator=g, dtype=torch.float64).to(dev)
Kb = torch.rand(2, 17, 17, generator=g, dtype=torch.float64)
Kb = (Kb @ Kb.transpose(1, 2) + 17 * torch.eye(17, dtype=torch.float64)).to(dev)
rb = torch.rand(2, 17, generator=g, dtype=torch.float64).to(dev)
for name, fn in [("gram_w", lambda: gram(pan, w=v).clone()),
                 ("xtv", lambda: gemv.xtv(pan, pan.xcols, v, grp, 2)),
                 ("xv", lambda: gemv.xv(pan, pan.xcols, V, grp)),
                 ("spd", lambda: spd_solve(Kb, rb)),
                 ("sum", lambda: (masks.double() * v).sum(1)),
                 ("amin", lambda: torch.where(masks[0], v, torch.full_like(v, 9.0)).amin())]:
    print(name, [h(fn()) for _ in range(3)], flush=True)
