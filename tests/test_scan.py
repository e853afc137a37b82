"""Lookback-free exclusive scan / compaction (csrc/scan.hip, ops/scan.py) against torch."""
import pytest
import torch

from ate_replication_causalml_amd.ops.scan import compact_rows, exclusive_cumsum


def test_scan_cpu_matches_torch():
    g = torch.Generator().manual_seed(0)
    for dt in (torch.int32, torch.int64):
        x = torch.randint(0, 7, (5000,), generator=g, dtype=dt)
        out, tot = exclusive_cumsum(x, total=True)
        assert out.dtype == dt
        assert torch.equal(out, torch.cumsum(x, 0, dtype=dt) - x)
        assert int(tot) == int(x.sum())
    m = torch.rand(777, generator=g) < 0.4
    assert torch.equal(compact_rows(m), torch.nonzero(m).flatten())


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 63, 4096, 4097, 100_003, 3_000_001])
@pytest.mark.parametrize("dt", [torch.int32, torch.int64])
def test_scan_gpu_matches_torch(gpu, n, dt):
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(n)
    x = torch.randint(0, 1000, (n,), generator=g, device=dev, dtype=dt)
    out, tot = exclusive_cumsum(x, total=True)
    ref = torch.cumsum(x, 0, dtype=dt) - x
    assert torch.equal(out, ref)
    assert int(tot.item()) == int(x.sum().item())


@pytest.mark.gpu
@pytest.mark.parametrize("n,p", [(1, 0.5), (5000, 0.0), (5000, 1.0), (2_000_003, 0.37)])
def test_compact_rows_gpu_matches_nonzero(gpu, n, p):
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(7)
    m = torch.rand(n, generator=g, device=dev) < p
    assert torch.equal(compact_rows(m), torch.nonzero(m).flatten())
