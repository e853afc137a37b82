"""K02 column moments / R scale() and K21 interaction expansion (ops/prep.py): CPU
formulas vs numpy, and the HIP kernels (csrc/prep.hip) vs the fp64 CPU path."""
import numpy as np
import pytest
import torch

from ate_replication_causalml_amd.data.dgp import r_scale as np_r_scale
from ate_replication_causalml_amd.ops import prep


def _x(n=1000, p=7, seed=0, nan=False):
    r = np.random.default_rng(seed)
    X = r.normal(size=(n, p)) * r.uniform(0.5, 5, size=p) + r.uniform(-3, 3, size=p)
    if nan:
        X[r.random((n, p)) < 0.02] = np.nan
    return X


def test_col_moments_cpu_matches_numpy():
    X = _x(nan=True)
    m = prep.col_moments(torch.as_tensor(X)).numpy()
    np.testing.assert_allclose(m[:, 0], (~np.isnan(X)).sum(0))
    np.testing.assert_allclose(m[:, 1], np.nanmean(X, 0), rtol=1e-13)
    np.testing.assert_allclose(m[:, 2], np.nanstd(X, 0, ddof=1), rtol=1e-12)


def test_r_scale_cpu_matches_dgp_scale():
    X = _x()
    np.testing.assert_allclose(prep.r_scale(torch.as_tensor(X)).numpy(), np_r_scale(X),
                               rtol=1e-12, atol=1e-12)
    part = prep.r_scale(torch.as_tensor(X), cols=[0, 3]).numpy()
    np.testing.assert_array_equal(part[:, 1], X[:, 1])


def test_interactions_cpu_layout():
    X = _x(50, 4)
    Z = prep.interactions(torch.as_tensor(X)).numpy()
    assert Z.shape == (50, 4 + 16)
    np.testing.assert_array_equal(Z[:, :4], X)
    np.testing.assert_allclose(Z[:, 4 + 2 * 4 + 3], X[:, 2] * X[:, 3])


@pytest.mark.gpu
def test_prep_kernels_match_cpu(gpu):
    X = _x(20000, 9, nan=True)
    m_cpu = prep.col_moments(torch.as_tensor(X)).numpy()
    m_gpu = prep.col_moments(torch.as_tensor(X, device=gpu)).cpu().numpy()
    np.testing.assert_allclose(m_gpu, m_cpu, rtol=1e-12)
    Xs = _x(20000, 9)
    s_cpu = prep.r_scale(torch.as_tensor(Xs), cols=[0, 1, 2, 5]).numpy()
    s_gpu = prep.r_scale(torch.as_tensor(Xs, device=gpu), cols=[0, 1, 2, 5]).cpu().numpy()
    np.testing.assert_allclose(s_gpu, s_cpu, rtol=1e-12, atol=1e-12)
    Z_cpu = prep.interactions(torch.as_tensor(Xs[:, :5])).numpy()
    Z_gpu = prep.interactions(torch.as_tensor(Xs[:, :5], device=gpu)).cpu().numpy()
    np.testing.assert_array_equal(Z_gpu, Z_cpu)


@pytest.mark.gpu
def test_loader_device_scale_matches_host(gpu, tmp_path):
    import pandas as pd
    from ate_replication_causalml_amd.data.dgp import BIN_NAMES, CTS_NAMES
    from ate_replication_causalml_amd.data.loader import OUTCOME, TREATMENT, load_social_pressure
    r = np.random.default_rng(4)
    n = 3000
    df = pd.DataFrame({c: r.normal(size=n) * 7 + 3 for c in CTS_NAMES})
    for c in BIN_NAMES:
        df[c] = (r.random(n) < 0.4).astype(float)
    df[OUTCOME] = (r.random(n) < 0.3).astype(float)
    df[TREATMENT] = (r.random(n) < 0.2).astype(float)
    df.loc[5, CTS_NAMES[2]] = np.nan
    f = tmp_path / "gotv.csv"
    df.to_csv(f, index=False)
    a = load_social_pressure(f, n_obs=2500)
    b = load_social_pressure(f, n_obs=2500, device=gpu)
    np.testing.assert_allclose(b.X, a.X, rtol=1e-12, atol=1e-12)
    np.testing.assert_array_equal(b.Y, a.Y)
