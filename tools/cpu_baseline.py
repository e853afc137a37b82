"""CPU comparison point for the headline metric (BASELINE.md "Measured CPU comparison point").

The reference publishes no throughput; BASELINE.md fixes the host CPU running this
framework's float64 reference path as the "other hardware". This measures, on the bench
panel shape (p=500, 5 folds), the two parts of one DML-PLR cross-fit on the CPU:

  * the per-fold Gram stack (the only O(N) part): torch BLAS on all host cores, fp64 and
    fp32, timed at N=2e5 and scaled linearly to N=1e7;
  * the CV-LASSO path solves + selection + residual pass (N-independent solves),
    reference/glmnet.py coordinate descent (Python), timed once.

  python tools/cpu_baseline.py [--rows 2e5] [--threads 8] > profiles/r02_cpu_baseline.json

rows/s of a full fit at N=1e7 and, as the conservative comparison, of the fp32 Gram ALONE
(no CPU implementation of the step can beat its own Gram on this host).
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=float, default=2e5)
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 8)
    a = ap.parse_args()
    import torch
    torch.set_num_threads(a.threads)
    from ate_replication_causalml_amd.data.device_dgp import synthetic_panel
    from ate_replication_causalml_amd.estimators.lasso import dml_phases
    from ate_replication_causalml_amd.ops.gram import gram

    n, N = int(a.rows), 10_000_000
    pan = synthetic_panel(n, p=500, folds=5, seed=1991, dtype="f64", device="cpu")
    out = {"host_threads": a.threads, "rows_timed": n, "p": 500, "folds": 5}
    for tag, dt in (("f64", torch.float64), ("f32", torch.float32)):
        X = pan.data.to(dt)
        best = 1e9
        for _ in range(3):
            t = time.perf_counter()
            for (r0, r1) in pan.seg_bounds:
                Xs = X[:, r0:r1]
                Xs @ Xs.T
            best = min(best, time.perf_counter() - t)
        out[f"gram_{tag}_s_per_1e7_rows"] = best * N / n
    ph = dml_phases(pan, 5, "min")
    st = ph[0](None)
    t = time.perf_counter()
    st = ph[1](st)
    st = ph[2](st)
    out["paths_resid_s"] = time.perf_counter() - t
    full = out["gram_f64_s_per_1e7_rows"] + out["paths_resid_s"]
    out["full_fit_s_at_1e7"] = full
    out["rows_per_s_full_fit"] = N / full
    out["rows_per_s_gram_f32_bound"] = N / out["gram_f32_s_per_1e7_rows"]
    out["note"] = ("CPU float64 reference path of this framework on the build host; the Gram "
                   "scales linearly in N (timed at rows_timed); the path solves do not depend "
                   "on N. rows_per_s_gram_f32_bound is an upper bound for any CPU "
                   "implementation of the step on this host.")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
