"""The multi-GPU bench step on one MI355X: device phases AND the RCCL all-reduces
captured in ONE hipGraph (utils/graphs.SegmentedStep), two fits in flight on two streams
with private Gram workspaces; the eager-collective fallback (graph segments with RCCL
between them) too. RCCL is real (a world-1 ``nccl`` process group); the communicator
reports world 2 so the collectives are in the step."""
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu


class _WideComm:
    """Real RCCL collectives on a 1-rank group, reported as world 2 so dml_phases inserts
    the C01 / C06 all-reduce phases (a sum over one rank is the identity)."""
    rank = 0
    world_size = 2

    def __init__(self, inner):
        self.inner = inner
        self.capturable = inner.capturable

    def all_reduce_(self, t):
        return self.inner.all_reduce_(t)

    def all_reduce_min_(self, t):
        return self.inner.all_reduce_min_(t)

    def barrier(self):
        self.inner.barrier()


@pytest.fixture(scope="module")
def rccl(gpu):
    import torch.distributed as dist
    from ate_replication_causalml_amd.parallel.comm import TorchComm
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0,
                            world_size=1, device_id=gpu)
    yield _WideComm(TorchComm())
    dist.destroy_process_group()


@pytest.mark.parametrize("capture_cc,slot_comms", [(True, False), (False, False), (True, True)])
def test_segmented_graphs_with_rccl_match_eager(gpu, rccl, capture_cc, slot_comms):
    from ate_replication_causalml_amd.data.device_dgp import synthetic_panel
    from ate_replication_causalml_amd.estimators.lasso import dml_crossfit_panel, dml_phases
    from ate_replication_causalml_amd.ops import gram as gram_op
    from ate_replication_causalml_amd.utils.graphs import Collective, SegmentedStep
    import numpy as np
    assert rccl.capturable
    pan = synthetic_panel(100000, p=500, folds=5, seed=4, dtype="bf16", device=gpu)
    seg = np.asarray(pan.seg_nreal, dtype=np.float64)
    want = dml_crossfit_panel(pan, 5, "min")[0].clone()
    runs = []
    comms = [rccl, rccl]
    if slot_comms:
        # bench.py at world > 1: one RCCL communicator per in-flight fit (dist.new_group),
        # so two fits' captured collectives never share a communicator
        import torch.distributed as dist
        from ate_replication_causalml_amd.parallel.comm import TorchComm
        comms = [rccl, _WideComm(TorchComm(dist.new_group([0])))]
        comms[1].barrier()
    for i in range(2):
        with gram_op.plan_slot(i):
            # the real group has one rank: every fold's paths must be solved here
            ph = dml_phases(pan, 5, "min", comm=comms[i], seg_counts=seg, shard_paths=False)
            assert sum(isinstance(p, Collective) and p.capturable for p in ph) == 2
            runs.append(SegmentedStep(ph, graph=True, capture_collectives=capture_cc))
    assert all(r.graphed for r in runs)
    if capture_cc:
        # the whole world-"2" step, both all-reduces included, is ONE graph launch
        assert all(r.collectives_captured and r.graph_count == 1 for r in runs), \
            [r.fallback_reason for r in runs]
    else:
        assert all(not r.collectives_captured and r.graph_count == 3 for r in runs)
    streams = [torch.cuda.Stream(gpu) for _ in runs]
    outs = [None, None]
    for k in range(6):
        with torch.cuda.stream(streams[k % 2]):
            outs[k % 2] = runs[k % 2]()["res"]
    torch.cuda.synchronize()
    assert outs[0].data_ptr() != outs[1].data_ptr()
    for o in outs:
        torch.testing.assert_close(o, want, rtol=0, atol=0)


def test_dist_estimators_single_graph_with_rccl(gpu, rccl):
    """Row-sharded / tree-parallel public estimators over RCCL run as ONE captured graph
    per call after the first (their all-reduces inside the graph) and equal their eager
    path. The comm reports world 2 (rank 0 holds the first half of the rows / trees; the
    sum over the single real rank is the identity), so every collective is issued."""
    import numpy as np
    from ate_replication_causalml_amd.estimators import forest as DF, lasso as DL, linear as DLin
    from ate_replication_causalml_amd.parallel.dist import DistContext
    rs = np.random.RandomState(11)
    n, p = 4000, 10
    d = DistContext(rccl, 0, n)
    assert d.capturable and d.n_local == n // 2
    for rep in range(3):
        X = rs.randn(n, p)
        W = (rs.rand(n) < 1 / (1 + np.exp(-X[:, 0]))).astype(float)
        Y = (rs.rand(n) < 1 / (1 + np.exp(-(X[:, 1] + 0.4 * W)))).astype(float)
        h = d.n_local
        for name, fn in (("dml", lambda g: DL.dml_plr_lasso(Y[:h], W[:h], X[:h], device=gpu,
                                                             dist=d, graph=g)),
                         ("aipw_glm", lambda g: DLin.aipw_glm(Y[:h], W[:h], X[:h], device=gpu,
                                                               dist=d, graph=g)),
                         ("lasso_single", lambda g: DL.lasso_single(Y[:h], W[:h], X[:h],
                                                                     device=gpu, dist=d, graph=g)),
                         ("aipw_rf", lambda g: DF.aipw_rf(Y, W, X, num_trees=40, device=gpu,
                                                          comm=rccl, graph=g))):
            e = fn(False)
            g = fn(True)
            assert g.diagnostics.get("hipgraph") is (rep > 0), (name, g.diagnostics)
            assert abs(g.ate - e.ate) < 1e-12, name
            if e.se is not None and e.se == e.se:        # LASSO rows have no SE (NaN)
                assert abs(g.se - e.se) < 1e-12, name


def test_ate_dml_single_graph_launch(gpu):
    """ate_dml on a GPU: the first call of a layout runs eagerly, the second captures the
    whole cross-fit, later calls on data of the same layout replay it (one graph launch);
    every call equals the eager estimator."""
    import numpy as np
    from ate_replication_causalml_amd.estimators import lasso as DL
    rs = np.random.RandomState(3)
    n, p = 4000, 12
    outs = []
    for rep in range(4):
        X = rs.randn(n, p)
        W = (rs.rand(n) < 1 / (1 + np.exp(-X[:, 0]))).astype(float)
        Y = X[:, 1] + 0.3 * W + rs.randn(n)
        eager = DL.dml_plr_lasso(Y, W, X, device=gpu, graph=False)
        graphed = DL.dml_plr_lasso(Y, W, X, device=gpu, graph=True)
        assert graphed.diagnostics.get("hipgraph") is (rep > 0)
        assert abs(graphed.ate - eager.ate) < 1e-12 and abs(graphed.se - eager.se) < 1e-12
        outs.append(graphed.ate)
    assert len(set(outs)) == 4          # the replays saw the new data
