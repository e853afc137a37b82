"""Public API, R-style API, replicate() with checkpoint/resume, CLI, logging/tracing."""
import json

import numpy as np
import pytest

import ate_replication_causalml_amd as ate
from ate_replication_causalml_amd import rstyle
from ate_replication_causalml_amd.config import ReplicateConfig, RunConfig

FAST = ReplicateConfig(n_obs=4000, dr_trees=30, dml_trees=20, cf_trees=30,
                       include=("oracle", "naive", "Direct Method", "Propensity_Weighting",
                                "Propensity_Regression", "Doubly Robust with logistic regression PS",
                                "Doubly Robust with Random Forest PS", "Causal Forest(GRF)"),
                       run=RunConfig(backend="cpu"))


def test_replicate_rows_and_labels():
    rep = ate.replicate(config=FAST)
    from ate_replication_causalml_amd.config import METHODS
    assert [r.method for r in rep.results] == [m for m in METHODS if m in FAST.include]
    assert rep.n_dropped > 0 and rep.n_mod + rep.n_dropped == 4000
    assert "Method" in rep.frame().columns and "oracle" in rep.table()


def test_replicate_checkpoint_resume(tmp_path):
    a = ate.replicate(config=FAST, checkpoint_dir=tmp_path)
    files = list(tmp_path.glob("*.npz"))
    assert len(files) == len(FAST.include)
    b = ate.replicate(config=FAST, checkpoint_dir=tmp_path)     # all rows from the cache
    for x, y in zip(a.results, b.results):
        assert (x.method, x.ate, x.se) == (y.method, y.ate, y.se)
    assert all(v < 0.05 for k, v in b.seconds.items() if k in FAST.include)


def test_reference_backend_matches_cpu_backend(tutorial):
    _, m, _ = tutorial
    ref = RunConfig(backend="reference")
    cpu = RunConfig(backend="cpu")
    for f in (lambda r: ate.ate_ols(m.Y, m.W, m.X, run=r),
              lambda r: ate.ate_aipw_glm(m.Y, m.W, m.X, run=r),
              lambda r: ate.ate_lasso_single(m.Y, m.W, m.X, run=r)):
        a, b = f(ref), f(cpu)
        assert a.ate == pytest.approx(b.ate, abs=1e-9)


def test_rstyle_dataframe_api(tutorial):
    d, m, _ = tutorial
    df = d.to_frame()
    out = rstyle.naive_ate(df, "W", "Y", method="oracle", run=RunConfig(backend="cpu"))
    assert list(out.columns) == ["Method", "ATE", "lower_ci", "upper_ci"]
    assert out.Method[0] == "oracle"
    p = rstyle.prop_score_lasso(df, "W", run=RunConfig(backend="reference"))
    assert p.shape == (len(df), 1)
    r = rstyle.double_ml(df, "W", "Y", num_tree=10, run=RunConfig(backend="cpu"))
    assert np.isfinite(r.ATE[0])


def test_jsonl_logging_and_tracing(tmp_path):
    from ate_replication_causalml_amd.utils import tracing
    from ate_replication_causalml_amd.utils.logging import read_jsonl, write_jsonl
    tracing.reset()
    rep = ate.replicate(config=FAST.with_(include=("oracle", "naive")))
    write_jsonl(tmp_path / "r.jsonl", rep.results, tag="t")
    recs = read_jsonl(tmp_path / "r.jsonl")
    assert [r["method"] for r in recs] == ["oracle", "naive"] and recs[0]["meta"]["tag"] == "t"
    assert any(s.name.startswith("ate_naive") for s in tracing.TRACE)
    tracing.export_jsonl(tmp_path / "t.jsonl")
    assert json.loads((tmp_path / "t.jsonl").read_text().splitlines()[0])["wall_ms"] >= 0


def test_cli_replicate(tmp_path, capsys):
    from ate_replication_causalml_amd.cli import main
    rc = main(["replicate", "--n-obs", "3000", "--backend", "cpu", "--only", "oracle", "naive",
               "--log", str(tmp_path / "x.jsonl"), "--plot", str(tmp_path / "p.png")])
    assert rc == 0 and (tmp_path / "p.png").exists()
    assert "oracle" in capsys.readouterr().out


def test_cli_dml_repeated(capsys):
    """`dml --repeats 3`: three distinct partitions of 25 micro-segments, median-aggregated;
    the aggregate is the median split ATE."""
    import json
    from ate_replication_causalml_amd.cli import main
    rc = main(["dml", "--n", "12000", "--p", "24", "--dtype", "f64", "--repeats", "3"])
    out = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert rc == 0 and out["repeats"] == 3 and len(out["splits"]) == 3
    assert out["ate"] == sorted(s[0] for s in out["splits"])[1]


def test_loader_reads_social_pressure_layout(tmp_path):
    """The CSV loader on a synthetic file with the reference's column names."""
    import pandas as pd
    from ate_replication_causalml_amd.data.dgp import BIN_NAMES, CTS_NAMES
    from ate_replication_causalml_amd.data.loader import load_social_pressure
    r = np.random.default_rng(0)
    n = 500
    df = pd.DataFrame({c: r.normal(size=n) for c in CTS_NAMES})
    for c in BIN_NAMES:
        df[c] = r.integers(0, 2, n)
    df["outcome_voted"] = r.integers(0, 2, n)
    df["treat_neighbors"] = r.integers(0, 2, n)
    df.loc[3, "city"] = np.nan
    path = tmp_path / "social.csv"
    df.to_csv(path, index=False)
    d = load_social_pressure(path, n_obs=400, seed=1)
    assert d.X.shape == (399, 21) or d.X.shape == (400, 21)
    assert np.allclose(d.X[:, :15].mean(0), 0, atol=0.2)


def test_rstyle_helpers_tau_hat_dr_est_and_chernozhukov():
    """The reference's two helpers (E10 tau_hat_dr_est, E12 chernozhukov) by name: one
    bootstrap replicate equals replicate b of the float64 oracle's bootstrap; one DML half
    equals the oracle's."""
    import numpy as np
    import pandas as pd
    from ate_replication_causalml_amd import rstyle
    from ate_replication_causalml_amd.config import RunConfig
    from ate_replication_causalml_amd.reference import estimators as R
    rs = np.random.RandomState(0)
    n = 400
    w = (rs.rand(n) < .5).astype(float)
    y = (rs.rand(n) < .4).astype(float)
    p = np.clip(rs.rand(n), .1, .9)
    m0, m1 = rs.rand(n), rs.rand(n)
    taus = [rstyle.tau_hat_dr_est(w, y, p, m0, m1, b=b) for b in range(4)]
    np.testing.assert_allclose(taus, R.aipw_bootstrap(w, y, p, m0, m1, B=4)[1], rtol=1e-12)
    X = rs.randn(n, 4)
    df = pd.DataFrame(X, columns=list("abcd"))
    df["W"], df["Y"] = w, y
    got = rstyle.chernozhukov(df, "W", "Y", np.arange(200), np.arange(200, n), 15,
                              run=RunConfig(backend="cpu"))
    want = R.chernozhukov(y, w, X, np.arange(200), np.arange(200, n), 15)
    assert got["tau_hat"] == want[0] and got["se_hat"] == want[1]
