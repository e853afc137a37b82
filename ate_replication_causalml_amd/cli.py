"""Command line: ``python -m ate_replication_causalml_amd <command>``.

  replicate  run the 14-row driver (ate_replication.Rmd) and print/log/plot it
  dml        K-fold DML cross-fit on a synthetic N x p panel (the north-star job)
  build      compile the gfx950 HIP library and the host C++ library
"""
from __future__ import annotations

import argparse
import json
import sys


def _replicate(a):
    from .api import replicate
    from .config import ReplicateConfig, RunConfig
    from .utils import tracing
    data = None
    if a.csv:
        from .data.loader import load_social_pressure
        data = load_social_pressure(a.csv, a.n_obs, a.seed)
    cfg = ReplicateConfig(n_obs=a.n_obs, dr_trees=a.dr_trees, dml_trees=a.dml_trees,
                          cf_trees=a.cf_trees, bootstrap_se=a.bootstrap_se,
                          include=tuple(a.only) if a.only else None,
                          run=RunConfig(backend=a.backend, dtype=a.dtype, compat=a.compat,
                                        seed=a.seed))
    rep = replicate(data, cfg, log_path=a.log, plot_path=a.plot, verbose=a.verbose,
                    checkpoint_dir=a.checkpoint)
    print(f"rows dropped by selection bias: {rep.n_dropped}  (df_mod n={rep.n_mod})")
    print(rep.table())
    if a.trace:
        tracing.export_jsonl(a.trace)
    if a.json:
        print(json.dumps({"seconds": rep.seconds}))
    return 0


def _dml(a):
    import torch
    from .data.device_dgp import synthetic_panel
    from .estimators.lasso import dml_crossfit_panel, dml_repeated_panel
    from .estimators.common import read_result
    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    if a.repeats > 1:
        # repeated cross-fitting: K*K micro-segments, `repeats` distinct K-fold partitions
        pan = synthetic_panel(a.n, p=a.p, folds=a.folds * a.folds, seed=a.seed, dtype=a.dtype,
                              device=dev)
        res, splits = dml_repeated_panel(pan, a.folds, a.repeats, a.lambda_rule,
                                         aggregate=a.aggregate)
        r = read_result(res, "DML cross-fit (LASSO, repeated)", n=a.n)
        out = {"ate": r.ate, "se": r.se, "lower_ci": r.lower_ci, "upper_ci": r.upper_ci,
               "repeats": a.repeats, "splits": splits.cpu().tolist()}
    else:
        pan = synthetic_panel(a.n, p=a.p, folds=a.folds, seed=a.seed, dtype=a.dtype, device=dev)
        res, mom, cv = dml_crossfit_panel(pan, a.folds, a.lambda_rule)
        r = read_result(res, "DML cross-fit (LASSO)", n=a.n)
        out = {"ate": r.ate, "se": r.se, "lower_ci": r.lower_ci, "upper_ci": r.upper_ci}
    print(json.dumps(out))
    return 0


def _build(a):
    from . import _build as b
    b.build_all()
    print("built")
    return 0


def main(argv=None):
    ap = argparse.ArgumentParser(prog="ate_replication_causalml_amd")
    sub = ap.add_subparsers(dest="cmd", required=True)
    r = sub.add_parser("replicate")
    r.add_argument("--csv", help="socialpresswgeooneperhh_NEIGH.csv (else synthetic DGP)")
    r.add_argument("--n-obs", type=int, default=50000)
    r.add_argument("--seed", type=int, default=1991)
    r.add_argument("--backend", default="auto", choices=["auto", "gpu", "cpu", "reference"])
    r.add_argument("--dtype", default="f64", choices=["f64", "f32", "bf16"])
    r.add_argument("--compat", default="reference", choices=["reference", "textbook"])
    r.add_argument("--dr-trees", type=int, default=2500)
    r.add_argument("--dml-trees", type=int, default=2000)
    r.add_argument("--cf-trees", type=int, default=2000)
    r.add_argument("--bootstrap-se", action="store_true")
    r.add_argument("--only", nargs="*", help="subset of method labels")
    r.add_argument("--log", help="append results as JSONL")
    r.add_argument("--plot", help="write the pointrange plot (png)")
    r.add_argument("--trace", help="append tracing spans as JSONL")
    r.add_argument("--checkpoint", help="directory for per-row results (resume)")
    r.add_argument("--json", action="store_true")
    r.add_argument("-v", "--verbose", action="store_true")
    r.set_defaults(fn=_replicate)
    d = sub.add_parser("dml")
    d.add_argument("--n", type=int, default=1_000_000)
    d.add_argument("--p", type=int, default=500)
    d.add_argument("--folds", type=int, default=5)
    d.add_argument("--dtype", default="bf16")
    d.add_argument("--seed", type=int, default=7)
    d.add_argument("--lambda-rule", default="min", choices=["min", "1se"])
    d.add_argument("--repeats", type=int, default=1,
                   help="> 1: repeated cross-fitting over that many distinct K-fold partitions")
    d.add_argument("--aggregate", default="median", choices=["median", "mean"])
    d.set_defaults(fn=_dml)
    b = sub.add_parser("build")
    b.set_defaults(fn=_build)
    a = ap.parse_args(argv)
    return a.fn(a)


if __name__ == "__main__":
    sys.exit(main())
