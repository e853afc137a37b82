"""CPU checks of the layout helpers behind two round-6 GPU paths:

* the one-byte Gram columns (data/device_dgp.byte_column_order, csrc/gram.hip BYTES): the
  columns the generator marks binary really hold only 0 / 1 (on the host twin of the
  device generator), and the physical order puts every one of them past BYTE_COL0 when the
  panel has the P = 512 shape;
* the fused GBDT root pass's row ranges (models/gbdt._two_ranges, csrc/gbdt.hip
  gbdt_hist2_kernel<ranges>)."""
import numpy as np
import pytest
import torch

from ate_replication_causalml_amd.data import device_dgp as D
from ate_replication_causalml_amd.models import gbdt as G


@pytest.mark.parametrize("dgp", ["tutorial", "rct"])
def test_binary_columns_are_zero_one(dgp):
    pan = D.synthetic_panel(3000, p=60, folds=5, seed=4, dtype="f64", device="cpu", dgp=dgp)
    X = pan.colmajor()
    for nm in D._binary_names(60):
        if nm in pan.cols:
            v = X[pan.cols[nm]][: pan.n]
            assert torch.all((v == 0) | (v == 1)), nm


def test_byte_column_order_shape():
    p = 500
    names = ["one"] + [f"x{j}" for j in range(p)] + ["W", "Y", "W_hi", "W_lo", "Y_hi", "Y_lo"]
    order = D.byte_column_order(names, p, 512)
    assert sorted(order) == sorted(names)
    binary = D._binary_names(p)
    assert all(nm in binary for nm in order[D.BYTE_COL0:])
    # the continuous columns come first, in generator order
    cont = [nm for nm in order if nm not in binary]
    assert cont == [nm for nm in names if nm not in binary] and len(cont) <= D.BYTE_COL0
    assert D.byte_column_order(names[:30], 23, 128) is None      # not the P = 512 shape


def test_two_ranges():
    t = lambda a: torch.as_tensor(np.asarray(a, dtype=np.int32))
    assert G._two_ranges(t(np.arange(10, 20))) == (10, 10, 20)
    assert G._two_ranges(t(np.r_[0:5, 9:14])) == (0, 5, 9)
    assert G._two_ranges(t(np.r_[0:5, 9:14, 20:22])) == (0, -1, 0)
    assert G._two_ranges(t([])) == (0, -1, 0)
    # every position maps to its row
    rows = np.r_[3:40, 77:100]
    a0, n0, a1 = G._two_ranges(t(rows))
    q = np.arange(len(rows))
    assert np.array_equal(np.where(q < n0, a0 + q, a1 + q - n0), rows)
