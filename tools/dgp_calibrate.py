"""Calibrate the tutorial DGP (data/dgp.py TUTORIAL) against the published run.

Targets (ate_replication.md:118 and the three plots): 41,062 of 50,000 rows
dropped by the selection transform, oracle ~0.096, naive ~0.003, Propensity_Weighting
(logistic PS) 0.064 < oracle, Propensity_Weighting_LASSOPS 0.011 < Propensity_Weighting,
Double Machine Learning 0.052.

    python tools/dgp_calibrate.py                     # evaluate data/dgp.TUTORIAL
    python tools/dgp_calibrate.py --search            # coarse search over the free constants
All estimators run on the float64 CPU reference path (reference/estimators.py).
"""
import argparse
import dataclasses
import itertools
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from ate_replication_causalml_amd.data import dgp as D  # noqa: E402
from ate_replication_causalml_amd.data.selection import apply_selection_bias  # noqa: E402
from ate_replication_causalml_amd.reference import estimators as R  # noqa: E402


def evaluate(params, dml_trees=0, lasso=True, seed=1991):
    df = D.make_tutorial_data(50_000, seed=seed, params=params)
    mod, drop = apply_selection_bias(df)
    out = {"dropped": int(len(drop)), "kept": int(mod.n), "tau_true": df.tau_true,
           "oracle": R.naive(df.Y, df.W).ate, "naive": R.naive(mod.Y, mod.W).ate,
           "mean_Y": float(df.Y.mean()),
           "hist_means": [float(v) for v in df.X[:, 16:21].mean(0)]}
    p = R.propensity_logistic(mod.W, mod.X)
    out["ipw_logit"] = R.ipw(mod.Y, mod.W, mod.X, p).ate
    out["ols"] = R.ols(mod.Y, mod.W, mod.X).ate
    if lasso:
        pl = R.propensity_lasso(mod.W, mod.X)
        out["ipw_lasso"] = R.ipw(mod.Y, mod.W, mod.X, pl).ate
    if dml_trees:
        out["double_ml"] = R.double_ml(mod.Y, mod.W, mod.X, num_trees=dml_trees).ate
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--search", action="store_true")
    ap.add_argument("--dml-trees", type=int, default=0)
    a = ap.parse_args()
    if not a.search:
        print(json.dumps(evaluate(D.TUTORIAL, a.dml_trees)), flush=True)
        return
    # vote-history marginals like the real file's: g2000 ~0.85, g2002 ~0.8, p2000 ~0.25,
    # p2002 ~0.4, p2004 ~0.4 (thresholds in units of the history score's SD)
    from scipy.stats import norm
    margins = (0.85, 0.80, 0.25, 0.40, 0.40)
    for lat, icpt, bh, bl, tl in itertools.product([0.3, 0.4], [-1.8, -1.6], [0.3, 0.35],
                                                   [0.2, 0.35], [0.4, 0.45]):
        sd = (1 + lat ** 2 * (1 + D.TUTORIAL.yob_latent ** 2)) ** 0.5
        th = tuple(float(-norm.ppf(m) * sd) for m in margins)
        P = dataclasses.replace(D.TUTORIAL, hist_thresh=th, hist_latent=lat, intercept=icpt,
                                b_hist=(bh,) * 5, b_latent=bl, tau_logit=tl)
        r = evaluate(P, lasso=False)
        print(json.dumps({"latent": lat, "intercept": icpt, "b_hist": bh, "b_latent": bl,
                          "tau_logit": tl, "thresh": [round(v, 4) for v in th],
                          **{k: (round(v, 4) if isinstance(v, float) else v)
                             for k, v in r.items() if k != "hist_means"}}), flush=True)


if __name__ == "__main__":
    main()
