"""R-compatible RNG (parallel/rrng.py) against values R >= 3.6 prints (default
Mersenne-Twister, sample.kind "Rejection"), and the loader's R-order row sample."""
import numpy as np
import pytest

from ate_replication_causalml_amd.parallel.rrng import RRandom, r_sample_rows


@pytest.mark.parametrize("seed,want", [
    (1, [0.2655087, 0.3721239, 0.5728534]),     # set.seed(1); runif(3)
    (42, [0.9148060, 0.9370754, 0.2861395]),    # set.seed(42); runif(3)
    (123, [0.2875775]),                          # set.seed(123); runif(1)
])
def test_runif_matches_r(seed, want):
    assert np.allclose(RRandom(seed).runif(len(want)), want, atol=5e-8)


@pytest.mark.parametrize("seed,want", [
    (1, [9, 4, 7, 1, 2, 5, 3, 10, 6, 8]),       # set.seed(1); sample(1:10)
    (42, [1, 5, 10, 8, 2, 4, 6, 9, 7, 3]),
    (123, [3, 10, 2, 8, 6, 9, 1, 7, 5, 4]),
])
def test_sample_matches_r(seed, want):
    assert list(RRandom(seed).sample_int(10)) == want


def test_sample_rows_is_a_prefix_of_the_full_permutation():
    full = r_sample_rows(1000, 1000, 1991)
    assert sorted(full) == list(range(1000))
    assert np.array_equal(r_sample_rows(1000, 300, 1991), full[:300])


def test_loader_uses_r_sample_order(tmp_path):
    import pandas as pd
    from ate_replication_causalml_amd.data.dgp import BIN_NAMES, CTS_NAMES
    from ate_replication_causalml_amd.data.loader import OUTCOME, TREATMENT, load_social_pressure
    rs = np.random.RandomState(0)
    n = 400
    df = pd.DataFrame({c: rs.randn(n) for c in CTS_NAMES})
    for c in BIN_NAMES:
        df[c] = rs.randint(0, 2, n).astype(float)
    df[OUTCOME] = rs.randint(0, 2, n).astype(float)
    df[TREATMENT] = np.arange(n) % 2
    df["yob"] = np.arange(n, dtype=float)      # the first continuous column is the row id
    path = tmp_path / "sp.csv"
    df.to_csv(path, index=False)
    d = load_social_pressure(path, n_obs=100, seed=1991)
    take = r_sample_rows(n, 100, 1991).astype(float)
    yob = (take - take.mean()) / take.std(ddof=1)
    assert np.allclose(d.X[:, 0], yob)         # R's sampled order, then scale()
