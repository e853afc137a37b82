"""Work census of the bench's CV-LASSO path problems on the CPU (design study for the path
kernel, csrc/enet.hip): runs glmnet's covariance-mode coordinate descent (the float64
reference semantics of reference/glmnet.cd_solve) on the dumped fold Gram stack and
counts, per problem and lambda, the passes, the coordinate moves, the nonzero and
ever-active set sizes and the 64-coordinate blocks a pass has to visit.

  python tools/enet_sim.py DUMPDIR [--problems all|full|W|Y] [--json OUT]

DUMPDIR holds G.npy / meta.json from tools/dump_bench_gram.py (GPU box)."""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def standardise(Gt, xcols, one, ycol):
    n = Gt[one, one]
    sx = Gt[one, xcols] / n
    vx = np.diag(Gt)[xcols] / n - sx * sx
    ju = vx > 0
    xs = np.where(ju, np.sqrt(np.maximum(vx, 0)), 1.0)
    C = (Gt[np.ix_(xcols, xcols)] / n - np.outer(sx, sx)) / np.outer(xs, xs)
    my = Gt[one, ycol] / n
    sy = np.sqrt(Gt[ycol, ycol] / n - my * my)
    g = np.where(ju, (Gt[xcols, ycol] / n - sx * my) / (xs * sy), 0.0)
    return C, g, ju


def census(C, g, ju, lams=None, nlam=100, flmin=1e-4, thr=1e-7, B=64):
    """glmnet gaussian lasso path (alpha = 1, unit penalty factors) with counters."""
    p = len(g)
    g = g.copy()
    a = np.zeros(p)
    ever = np.zeros(p, dtype=bool)
    alf = flmin ** (1.0 / (nlam - 1)) if lams is None else 1.0
    rows = []
    alm = 0.0
    rsq_prev = rsq = 0.0
    full_idx = np.flatnonzero(ju)
    T = (p + B - 1) // B
    for m in range(nlam if lams is None else len(lams)):
        if lams is not None:
            alm = lams[m]
        elif m == 0:
            alm = 9.9e35
        elif m == 1:
            alm = alf * np.max(np.abs(g[ju]))
        else:
            alm *= alf
        st = dict(m=m, full=0, active=0, moves_full=0, moves_active=0, blocks_full=0,
                  blocks_active=0, dense_blocks=0, changed_full_blocks=[])
        while True:
            # full pass
            st["full"] += 1
            dlx = 0.0
            moved = []
            for j in full_idx:
                u = g[j] + a[j]
                if a[j] == 0.0 and abs(u) <= alm:
                    continue
                v = abs(u) - alm
                an = np.sign(u) * v if v > 0 else 0.0
                if an == a[j]:
                    continue
                d = an - a[j]
                rsq += d * (2 * g[j] - d)
                a[j] = an
                ever[j] = True
                dlx = max(dlx, d * d)
                g -= C[:, j] * d
                moved.append(j)
            st["moves_full"] += len(moved)
            st["blocks_full"] += T
            nzb = np.bincount(np.flatnonzero(a) // B, minlength=T)
            st["dense_blocks"] += int((nzb >= 56).sum())
            st["changed_full_blocks"].append(int(len(set(np.asarray(moved, int) // B))))
            if dlx < thr:
                break
            while True:
                st["active"] += 1
                dlx = 0.0
                act = np.flatnonzero(ever)
                st["blocks_active"] += len(set(act // B))
                for j in act:
                    u = g[j] + a[j]
                    v = abs(u) - alm
                    an = np.sign(u) * v if v > 0 else 0.0
                    if an == a[j]:
                        continue
                    d = an - a[j]
                    rsq += d * (2 * g[j] - d)
                    a[j] = an
                    dlx = max(dlx, d * d)
                    g -= C[:, j] * d
                    st["moves_active"] += 1
                if dlx < thr:
                    break
        st["nnz"] = int((a != 0).sum())
        st["ever"] = int(ever.sum())
        st["lam"] = alm
        rows.append(st)
        if lams is None and m >= 4:
            if rsq - rsq_prev < 1e-5 * rsq or rsq > 0.999:
                break
        rsq_prev = rsq
    lam_seq = [r["lam"] for r in rows]
    return rows, lam_seq


def summarise(name, rows):
    tot = lambda k: int(sum(r[k] for r in rows))  # noqa: E731
    return {"problem": name, "nlam": len(rows), "full_passes": tot("full"),
            "active_passes": tot("active"), "moves_full": tot("moves_full"),
            "moves_active": tot("moves_active"), "visits_full": tot("blocks_full"),
            "visits_active": tot("blocks_active"), "dense_block_visits": tot("dense_blocks"),
            "nnz_end": rows[-1]["nnz"], "ever_end": rows[-1]["ever"],
            "nnz_q": [rows[int(f * (len(rows) - 1))]["nnz"] for f in (0.1, 0.25, 0.5, 0.75, 1.0)],
            "ever_q": [rows[int(f * (len(rows) - 1))]["ever"] for f in (0.1, 0.25, 0.5, 0.75, 1.0)]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dump")
    ap.add_argument("--problems", default="full")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    G = np.load(os.path.join(a.dump, "G.npy"))
    meta = json.load(open(os.path.join(a.dump, "meta.json")))
    xcols, one = meta["xcols"], meta["one"]
    nseg = G.shape[0]
    out = []
    for k in range(nseg if a.problems != "one" else 1):   # outer fold k: train on the others
        train = [s for s in range(nseg) if s != k]
        Gt = G[train].sum(0)
        for yname in ("Y", "W"):
            C, g, ju = standardise(Gt, xcols, one, meta[yname])
            rows, lam = census(C, g, ju)
            s = summarise(f"full k={k} {yname}", rows)
            print(json.dumps(s), flush=True)
            out.append(s)
            if a.problems == "all":
                for h in train:   # inner folds share the full problem's lambdas
                    Gf = G[[s2 for s2 in train if s2 != h]].sum(0)
                    Cf, gf, juf = standardise(Gf, xcols, one, meta[yname])
                    rf, _ = census(Cf, gf, juf, lams=lam)
                    sf = summarise(f"fold k={k} h={h} {yname}", rf)
                    print(json.dumps(sf), flush=True)
                    out.append(sf)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f)


if __name__ == "__main__":
    main()
