"""Measured throughput for the BASELINE.json configs on ONE device (bench.py covers the
headline metric). Each line is a JSON object with the config, its size and wall time;
configs whose named size needs 8 GPUs are run at the size given in "rows"/"p"
(stated in the output) — the multi-GPU paths are the same code with a communicator.

  2: DML ATE, LASSO nuisance, N=1e6 p=500 bf16
  3: AIPW ATE, random-forest nuisances, 5-fold cross-fit
  4: causal-forest ATE + 1000-replicate bootstrap SE
  5: DML ATE with histogram-GBDT nuisances
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# imported before the first CUDA call: the package sets its HIP hardware-queue default
import ate_replication_causalml_amd  # noqa: E402,F401


def _sync():
    import torch
    if torch.cuda.is_available():
        torch.cuda.synchronize()


def timed(fn, reps=1, warm=True):
    if warm:          # large configs: one cold run (first-call overheads included)
        fn()
    _sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        r = fn()
    _sync()
    return r, (time.perf_counter() - t0) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="2,3,4,5")
    ap.add_argument("--dgp", default="tutorial", choices=["tutorial", "rct"],
                    help="tutorial: the selection-biased df_mod at scale (panels: "
                         "synthetic_panel(dgp='tutorial'); host data: the kept rows of "
                         "data/panel_selection.selected_rows); rct: the unselected panels")
    ap.add_argument("--n3", type=int, default=200_000)
    ap.add_argument("--trees3", type=int, default=100)
    ap.add_argument("--n4", type=int, default=50_000)
    ap.add_argument("--n5", type=int, default=1_000_000)
    ap.add_argument("--p5", type=int, default=100)
    ap.add_argument("--trees5", type=int, default=50)
    ap.add_argument("--p3", type=int, default=100)
    ap.add_argument("--panel3", action="store_true",
                    help="config 3 from a device-generated bf16 panel (estimators/crossfit."
                         "aipw_rf_crossfit_panel; use --n3 10000000 --p3 500 --shard3 0/8 for "
                         "the per-GPU work of the 8-GPU config)")
    ap.add_argument("--shard3", default=None, help="rank/world tree shard on this device")
    ap.add_argument("--serial3", action="store_true",
                    help="config 3: grow the 15 forests one after another (each fills the GPU "
                         "on the level engine) instead of concurrently on streams")
    ap.add_argument("--panel5", action="store_true",
                    help="config 5 from a device-generated bf16 panel (use --n5 12500000 "
                         "--p5 2000 for the per-GPU shard of N=1e8)")
    a = ap.parse_args()
    import torch
    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    want = {int(c) for c in a.configs.split(",")}
    out = []
    if 2 in want:
        from ate_replication_causalml_amd.data.device_dgp import synthetic_panel
        from ate_replication_causalml_amd.estimators.lasso import dml_crossfit_panel
        pan = synthetic_panel(1_000_000, p=500, folds=5, seed=7, dtype="bf16", device=dev,
                              dgp=a.dgp)
        (res, _, _), s = timed(lambda: dml_crossfit_panel(pan, 5, "min"), reps=5)
        out.append({"config": 2, "estimator": "DML-PLR (CV-LASSO)", "rows": 1_000_000, "p": 500,
                    "dtype": "bf16", "seconds": s, "rows_per_s": 1e6 / s,
                    "ate": float(res[0]), "se": float(res[1])})
        print(json.dumps(out[-1]), flush=True)
        del pan
    if 3 in want or 4 in want or 5 in want:
        from ate_replication_causalml_amd.data.dgp import make_tutorial_data as _make
        from ate_replication_causalml_amd.data.panel_selection import selected_rows

        def make_tutorial_data(n, seed, p_extra=0):
            """host data of config 3/4/5: the tutorial's kept rows (df_mod) or the RCT"""
            if a.dgp == "tutorial":
                return selected_rows(n, seed, p_extra=p_extra, device=dev)[0]
            return _make(n, seed=seed, p_extra=p_extra)
    if 3 in want and a.panel3:
        from ate_replication_causalml_amd.data.device_dgp import synthetic_panel
        from ate_replication_causalml_amd.estimators.crossfit import aipw_rf_crossfit_panel
        pan = synthetic_panel(a.n3, p=a.p3, folds=5, seed=11, dtype="bf16", device=dev,
                              dgp=a.dgp)
        shard = tuple(int(v) for v in a.shard3.split("/")) if a.shard3 else None
        r, s = timed(lambda: aipw_rf_crossfit_panel(pan, num_trees=a.trees3, tree_shard=shard,
                                                    concurrent=not a.serial3),
                     warm=a.n3 <= 2_000_000)
        out.append({"config": 3, "estimator": "AIPW 5-fold cross-fit, RF nuisances (3 forests/"
                    "fold), HBM panel, device binning", "rows": a.n3, "p": a.p3,
                    "trees_per_forest": a.trees3, "tree_shard": a.shard3,
                    "trees_this_device": r.diagnostics.get("trees_this_device"),
                    "serial": a.serial3,
                    "seconds": s, "rows_per_s": a.n3 / s, "ate": r.ate, "se": r.se})
        print(json.dumps(out[-1]), flush=True)
        del pan
    elif 3 in want:
        from ate_replication_causalml_amd.estimators.crossfit import aipw_crossfit
        d = make_tutorial_data(a.n3, seed=11, p_extra=79)
        r, s = timed(lambda: aipw_crossfit(d.Y, d.W, d.X, folds=5, learner="rf",
                                           num_trees=a.trees3, device=dev))
        out.append({"config": 3, "estimator": "AIPW 5-fold cross-fit, RF nuisances (3 forests/fold)",
                    "rows": a.n3, "p": d.X.shape[1], "trees_per_forest": a.trees3,
                    "seconds": s, "rows_per_s": a.n3 / s, "ate": r.ate, "se": r.se})
        print(json.dumps(out[-1]), flush=True)
    if 4 in want:
        from ate_replication_causalml_amd.estimators.crossfit import causal_forest_bootstrap
        d = make_tutorial_data(a.n4, seed=12)
        r, s = timed(lambda: causal_forest_bootstrap(d.Y, d.W, d.X, num_trees=2000, B=1000,
                                                     device=dev))
        out.append({"config": 4, "estimator": "causal forest (2000 trees) + 1000 bootstrap reps",
                    "rows": a.n4, "p": d.X.shape[1], "seconds": s, "rows_per_s": a.n4 / s,
                    "ate": r.ate, "se": r.se})
        print(json.dumps(out[-1]), flush=True)
    if 5 in want and a.panel5:
        # per-GPU shard of the named config (N=1e8 over 8 GPUs, p=2000): panel generated
        # and binned in HBM (no host copy of X)
        from ate_replication_causalml_amd.data.device_dgp import synthetic_panel
        from ate_replication_causalml_amd.estimators.boosting import dml_plr_gbdt_panel
        pan = synthetic_panel(a.n5, p=a.p5, folds=5, seed=13, dtype="bf16", device=dev,
                              dgp=a.dgp)
        r, s = timed(lambda: dml_plr_gbdt_panel(pan, n_trees=a.trees5, depth=6))
        out.append({"config": 5, "estimator": "DML-PLR, GBDT nuisances (depth 6), HBM panel",
                    "rows": a.n5, "p": a.p5, "trees": a.trees5, "seconds": s,
                    "rows_per_s": a.n5 / s, "ate": r.ate, "se": r.se})
        print(json.dumps(out[-1]), flush=True)
        del pan
    elif 5 in want:
        from ate_replication_causalml_amd.estimators.boosting import dml_plr_gbdt
        d = make_tutorial_data(a.n5, seed=13, p_extra=a.p5 - 21)
        r, s = timed(lambda: dml_plr_gbdt(d.Y, d.W, d.X, folds=5, n_trees=a.trees5, depth=6,
                                          device=dev))
        out.append({"config": 5, "estimator": "DML-PLR, GBDT nuisances (depth 6)",
                    "rows": a.n5, "p": d.X.shape[1], "trees": a.trees5, "seconds": s,
                    "rows_per_s": a.n5 / s, "ate": r.ate, "se": r.se})
        print(json.dumps(out[-1]), flush=True)


if __name__ == "__main__":
    main()
