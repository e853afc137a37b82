"""Guards added after the round-1 review: truncated CV fold paths are loud,
Gram plans are bounded and survive eviction while a graph holds them, checkpoint keys
cover every byte, the segmented (graph + eager collective) DML step equals the eager one
on simulated ranks."""
import numpy as np
import pytest
import torch

from ate_replication_causalml_amd.ops import gram as gram_op
from ate_replication_causalml_amd.ops.enet import EnetCvResult, poison_if_truncated
from ate_replication_causalml_amd.utils import graphs
from ate_replication_causalml_amd.utils.checkpoint import fingerprint
from ate_replication_causalml_amd.utils.guards import NumericalError


def test_poison_if_truncated():
    a = torch.arange(4, dtype=torch.float64)
    ok = poison_if_truncated(torch.tensor([3, 5, 7], dtype=torch.int32), a)[0]
    torch.testing.assert_close(ok, a)
    bad = poison_if_truncated(torch.tensor([3, -1, 7], dtype=torch.int32), a)[0]
    assert torch.isnan(bad).all()


def test_cv_result_check_raises_on_truncated_fold():
    z = torch.zeros(1)
    r = EnetCvResult(z, z, z, z, z, z, z, z, [], torch.tensor([5]),
                     torch.tensor([4, -1, 6], dtype=torch.int32))
    with pytest.raises(NumericalError, match=r"\[1\]"):
        r.check()
    r.fold_npass = torch.tensor([4, 2, 6], dtype=torch.int32)
    assert r.check() is r


def test_lognet_cv_result_check():
    from ate_replication_causalml_amd.ops.lognet import LognetCvResult
    z = torch.zeros(1)
    r = LognetCvResult(z, z, z, z, z, z, z, z, torch.tensor([10, 4, -1, 3], dtype=torch.int32))
    with pytest.raises(NumericalError):
        r.check()


def _panel(n, seed):
    from ate_replication_causalml_amd.data.device_dgp import synthetic_panel
    return synthetic_panel(n, p=24, folds=5, seed=seed, dtype="f64", device="cpu")


def test_gram_plan_cache_is_bounded_and_pinned(monkeypatch):
    monkeypatch.setattr(gram_op, "PLAN_CACHE_MAX", 3)
    gram_op.clear_plans()
    pans = [_panel(2000 + 64 * i, i) for i in range(6)]
    first = gram_op.plan_for(pans[0])
    assert gram_op.plan_for(pans[0]) is first           # cache hit
    # a "capture" in progress pins what it touched
    prev, graphs._pins = graphs._pins, []
    try:
        pinned = gram_op.plan_for(pans[1])
        held = graphs._pins
    finally:
        graphs._pins = prev
    for p in pans[2:]:
        gram_op.plan_for(p)
    assert len(gram_op._plan_cache) == 3
    assert all(pl is not first for pl in gram_op._plan_cache.values())   # LRU evicted
    assert held == [pinned]          # the graph's reference keeps the evicted plan alive
    gram_op.clear_plans()
    assert not gram_op._plan_cache


def test_fingerprint_sees_every_element():
    a = np.random.RandomState(0).rand(200_000)
    b = a.copy()
    # an edit whose effect on the sum cancels, at an index a strided sample would skip
    b[12345] += 0.25
    b[54321] -= 0.25
    assert fingerprint(a) != fingerprint(b)
    assert fingerprint(a) == fingerprint(a.copy())


def test_segmented_step_matches_eager_on_simulated_ranks():
    """dml_phases under SegmentedStep (collectives between device phases) on 2 simulated
    ranks equals the single-process cross-fit on the concatenated data."""
    from ate_replication_causalml_amd.data.device_dgp import synthetic_panel
    from ate_replication_causalml_amd.estimators.lasso import dml_crossfit_panel, dml_phases
    from ate_replication_causalml_amd.parallel.comm import run_simulated

    n = 6000
    want = dml_crossfit_panel(synthetic_panel(n, p=24, folds=5, seed=3, dtype="f64",
                                              device="cpu"), 5)[0]

    def rank_fn(comm):
        pan = synthetic_panel(n, p=24, folds=5, seed=3, dtype="f64", device="cpu",
                              rank=comm.rank, world=comm.world_size)
        out = []
        for shard in (True, False):
            step = graphs.SegmentedStep(dml_phases(pan, 5, "min", comm=comm, shard_paths=shard),
                                        graph=False, warmup=0)
            # C01 Gram, C08 coefficients (sharded path solves only), C06 moments
            assert sum(isinstance(ph, graphs.Collective) for ph in step.phases) == 2 + shard
            out.append(step()["res"])
        return out

    got = run_simulated(2, rank_fn)
    for sharded, unsharded in got:
        torch.testing.assert_close(sharded, unsharded, rtol=0, atol=0)
        torch.testing.assert_close(sharded, want, rtol=1e-9, atol=1e-12)


def test_zeroed_views_share_one_buffer():
    """ops/enet._zeroed: the path kernel's zero-initialised outputs carved from one buffer
    (one fill launch), typed, shaped, zero, 256-B aligned and non-overlapping."""
    from ate_replication_causalml_amd.ops.enet import _zeroed
    specs = [((3, 5, 64), torch.float32), ((12, 100, 7), torch.float64), ((12, 100), torch.float64),
             ((12,), torch.int32), ((12,), torch.int32), ((12,), torch.int32)]
    ts = _zeroed(torch.device("cpu"), *specs)
    base = ts[0].untyped_storage().data_ptr()
    spans = []
    for t, (sh, dt) in zip(ts, specs):
        assert tuple(t.shape) == sh and t.dtype == dt and t.is_contiguous()
        assert bool((t == 0).all())
        assert t.untyped_storage().data_ptr() == base          # one allocation
        off = t.data_ptr() - base
        assert off % 256 == 0
        spans.append((off, off + t.numel() * t.element_size()))
    spans.sort()
    assert all(a[1] <= b[0] for a, b in zip(spans, spans[1:]))
