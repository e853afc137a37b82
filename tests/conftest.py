import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def tutorial():
    from ate_replication_causalml_amd.data.dgp import make_tutorial_data
    from ate_replication_causalml_amd.data.selection import apply_selection_bias
    d = make_tutorial_data(n=6000, seed=1991)
    m, drop = apply_selection_bias(d)
    return d, m, drop


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from ate_replication_causalml_amd import _native
    _native.hip()  # fail loudly if the kernel library is missing
    return torch.device("cuda:0")
