#!/usr/bin/env python3
"""Per-phase timing of the DML cross-fit step with HIP events (gram / CV-LASSO /
residual pass), plus an end-to-end step time. Usage: python tools/phase_timing.py --n 1e7 --p 500"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=float, default=1e7)
    ap.add_argument("--p", type=int, default=500)
    ap.add_argument("--folds", type=int, default=5)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import torch
    from ate_replication_causalml_amd.data.device_dgp import synthetic_panel
    from ate_replication_causalml_amd.estimators.lasso import dml_residual_moments
    from ate_replication_causalml_amd.ops import stats as S
    from ate_replication_causalml_amd.ops.enet import cv_enet_gaussian
    from ate_replication_causalml_amd.ops.gram import gram
    dev = torch.device("cuda:0")
    pan = synthetic_panel(int(args.n), p=args.p, folds=args.folds, seed=1991, dtype=args.dtype,
                          device=dev, dgp=os.environ.get("ATE_DGP", "tutorial"))
    K = args.folds
    full_sets = [[s for s in range(K) if s != k] for k in range(K)]
    ycols = [pan.cols["Y"], pan.cols["W"]]
    ev = lambda: torch.cuda.Event(enable_timing=True)
    out = {}
    for rep in range(args.reps + 1):
        e = [ev() for _ in range(4)]
        e[0].record()
        G = gram(pan)
        e[1].record()
        cv = cv_enet_gaussian(G, pan, pan.xcols, ycols, full_sets=full_sets)
        e[2].record()
        coef = cv.coef_min.reshape(K, 2, -1).contiguous()
        mom = dml_residual_moments(pan, coef)
        res = S.dml_finalize(mom, "plr")
        e[3].record()
        torch.cuda.synchronize()
        if rep:
            for name, (a, b) in {"gram": (0, 1), "cv_lasso": (1, 2), "resid": (2, 3),
                                 "total": (0, 3)}.items():
                out.setdefault(name, []).append(e[a].elapsed_time(e[b]))
    summary = {k: min(v) for k, v in out.items()}
    summary["npass_full"] = cv.npass.cpu().tolist()
    summary["nlam_full"] = cv.nlam.cpu().tolist()
    summary["ate_se"] = res.cpu().tolist()
    print(json.dumps(summary))


if __name__ == "__main__":
    main()
