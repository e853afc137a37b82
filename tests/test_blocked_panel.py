"""64-row blocked panel layout (ops/panel.py DevicePanel.blocked): the same values as the
column-major panel, the same Gram stack, the same DML cross-fit. The GPU test pins the
strided kernels (dgp fill, paired-tile bf16 Gram, bf16 residual pass) bit for bit against
the column-major panel."""
import numpy as np
import pytest
import torch


def _pair(device, n=3000, p=24, dtype="f64"):
    from ate_replication_causalml_amd.data.device_dgp import synthetic_panel
    a = synthetic_panel(n, p=p, folds=3, seed=5, dtype=dtype, device=device)
    b = synthetic_panel(n, p=p, folds=3, seed=5, dtype=dtype, device=device, blocked=True)
    return a, b


def test_blocked_panel_cpu_matches_colmajor():
    from ate_replication_causalml_amd.ops.gram import gram
    from ate_replication_causalml_amd.estimators.lasso import dml_crossfit_panel
    a, b = _pair("cpu")
    assert b.blocked and b.data.shape == (a.ld // 64, a.P, 64)
    assert (b.P, b.ld) == (a.P, a.ld)
    assert torch.equal(b.colmajor(), a.data)
    assert torch.equal(b.col("Y"), a.col("Y"))
    assert b.strides() == (64, 64 * a.P) and a.strides() == (a.ld, 64)
    torch.testing.assert_close(gram(b), gram(a), rtol=0, atol=0)
    ra = dml_crossfit_panel(a, 3, "min")[0]
    rb = dml_crossfit_panel(b, 3, "min")[0]
    torch.testing.assert_close(rb, ra, rtol=0, atol=0)


def test_blocked_panel_rejected_by_colmajor_kernels():
    a, b = _pair("cpu")
    assert a.cm_ld == a.ld
    with pytest.raises(NotImplementedError):
        b.cm_ld


@pytest.mark.gpu
def test_blocked_panel_gpu_bit_identical(gpu):
    from ate_replication_causalml_amd.ops.gram import gram
    from ate_replication_causalml_amd.estimators.lasso import dml_crossfit_panel
    a, b = _pair(gpu, n=200000, p=500, dtype="bf16")
    torch.cuda.synchronize()
    # the blocked GPU panel may keep its {0, 1} columns last (one-byte Gram path,
    # data/device_dgp.byte_column_order): compare column by name, padding after
    named = [b.cols[nm] for nm, _ in sorted(a.cols.items(), key=lambda kv: kv[1])]
    perm = named + [c for c in range(b.P) if c not in set(named)]
    perm = torch.tensor(perm, device=gpu)
    assert torch.equal(b.colmajor()[perm], a.data)
    Gb = gram(b).clone()
    torch.testing.assert_close(Gb[:, perm][:, :, perm], gram(a).clone(), rtol=0, atol=0)
    ra = dml_crossfit_panel(a, 3, "min")[0].clone()
    rb = dml_crossfit_panel(b, 3, "min")[0].clone()
    torch.testing.assert_close(rb, ra, rtol=0, atol=0)
    assert np.isfinite(ra.cpu().numpy()).all()
