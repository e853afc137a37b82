"""Distributed algorithms without a cluster: the in-process thread simulator and a
real 2-process gloo run must reproduce the world-size-1 DML result (sufficient
statistics are all-reduced; the data never moves)."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from ate_replication_causalml_amd.data.device_dgp import fold_slices, synthetic_panel
from ate_replication_causalml_amd.estimators.lasso import dml_crossfit_panel
from ate_replication_causalml_amd.parallel.comm import LocalComm, run_simulated

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_fold_slices_partition():
    n, K = 1000, 5
    for world in (1, 2, 3, 4, 8):
        rows = []
        for r in range(world):
            for g0, c in fold_slices(n, K, r, world):
                rows.extend(range(g0, g0 + c))
        assert sorted(rows) == list(range(n))


def _dml(world, rank, comm, n=1500, p=24):
    pan = synthetic_panel(n, p=p, folds=5, seed=3, dtype="f64", device="cpu", rank=rank,
                          world=world)
    res, mom, _ = dml_crossfit_panel(pan, 5, comm=comm)
    return res.numpy(), mom.numpy()


@pytest.mark.parametrize("world", [2, 4])
def test_thread_simulated_dml_matches_single(world):
    ref, mref = _dml(1, 0, LocalComm())
    outs = run_simulated(world, lambda c: _dml(world, c.rank, c))
    for res, mom in outs:
        assert np.allclose(res, ref, rtol=1e-9, atol=1e-12)
        assert np.allclose(mom, mref, rtol=1e-9)


def test_gloo_two_process_dml():
    script = r"""
import os, sys, json
sys.path.insert(0, %r)
import torch, torch.distributed as dist
dist.init_process_group("gloo")
from ate_replication_causalml_amd.parallel.comm import TorchComm
from ate_replication_causalml_amd.data.device_dgp import synthetic_panel
from ate_replication_causalml_amd.estimators.lasso import dml_crossfit_panel
c = TorchComm()
pan = synthetic_panel(1500, p=24, folds=5, seed=3, dtype="f64", device="cpu", rank=c.rank, world=c.world_size)
res, mom, _ = dml_crossfit_panel(pan, 5, comm=c)
if c.rank == 0:
    print("RESULT", json.dumps(res.tolist()))
dist.destroy_process_group()
""" % ROOT
    import tempfile
    with tempfile.NamedTemporaryFile("w", suffix=".py", delete=False) as f:
        f.write(script)
        path = f.name
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", "--master-port=29517", path]
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=300)
    finally:
        os.unlink(path)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("RESULT")][0]
    import json
    got = np.array(json.loads(line.split(" ", 1)[1]))
    ref, _ = _dml(1, 0, LocalComm())
    assert np.allclose(got, ref, rtol=1e-9)


def test_gloo_two_process_sharded_estimators():
    """Real torch.distributed (gloo) ranks: row-sharded AIPW-glm with sharded bootstrap,
    and a tree-parallel RF OOB propensity, equal to the single-process results."""
    script = r"""
import os, sys, json
sys.path.insert(0, %r)
import numpy as np, torch, torch.distributed as dist
dist.init_process_group("gloo")
from ate_replication_causalml_amd.parallel.comm import TorchComm
from ate_replication_causalml_amd.parallel.dist import DistContext
from ate_replication_causalml_amd.data.dgp import make_tutorial_data
from ate_replication_causalml_amd.data.selection import apply_selection_bias
from ate_replication_causalml_amd.estimators import linear as D
from ate_replication_causalml_amd.models import forest as F
c = TorchComm()
m, _ = apply_selection_bias(make_tutorial_data(4000, 1991))
d = DistContext.for_rank(c, len(m.Y))
r = D.aipw_glm(d.local(m.Y), d.local(m.W), d.local(m.X), bootstrap_se=True, B=30, device="cpu", dist=d)
fr = F.fit_forest_sharded(m.X, F.KIND_CLASS, 16, c, y=m.W, seed=4, backend="cpu")
p = F.predict_tree_parallel(fr, c, oob=True)
if c.rank == 0:
    print("RESULT", json.dumps([r.ate, r.se, float(np.nansum(p))]))
dist.destroy_process_group()
""" % ROOT
    import json
    import tempfile
    with tempfile.NamedTemporaryFile("w", suffix=".py", delete=False) as f:
        f.write(script)
        path = f.name
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", "--master-port=29519", path]
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=300)
    finally:
        os.unlink(path)
    assert r.returncode == 0, r.stderr[-3000:]
    got = json.loads([l for l in r.stdout.splitlines() if l.startswith("RESULT")][0].split(" ", 1)[1])
    from ate_replication_causalml_amd.data.dgp import make_tutorial_data
    from ate_replication_causalml_amd.data.selection import apply_selection_bias
    from ate_replication_causalml_amd.estimators import linear as D
    from ate_replication_causalml_amd.models import forest as F
    m, _ = apply_selection_bias(make_tutorial_data(4000, 1991))
    ref = D.aipw_glm(m.Y, m.W, m.X, bootstrap_se=True, B=30, device="cpu")
    p = F.rf_classifier(m.X, m.W, num_trees=16, seed=4, backend="cpu").oob_proba()
    assert got[0] == pytest.approx(ref.ate, rel=1e-9)
    assert got[1] == pytest.approx(ref.se, rel=1e-8)
    assert got[2] == pytest.approx(float(np.nansum(p)), rel=1e-12)


@pytest.mark.parametrize("world", [2, 6])
def test_bench_multi_rank_gloo_contract(world):
    """bench.py under torch.distributed.run (gloo ranks on the CPU): one JSON line from
    rank 0 with the driver's fields, weak scaling (rows per rank fixed), and the same
    ATE / SE as one process holding all the rows. World 6 > 5 folds: ranks 5.. solve no
    CV paths (the path solves are sharded by outer fold) and contribute zeros."""
    import json
    bench = os.path.join(ROOT, "bench.py")
    rows = 3000 if world == 2 else 1000
    args = ["--rows", str(rows), "--p", "24", "--dtype", "f64", "--steps", "1", "--warmup", "1"]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={world}", "--master-addr=127.0.0.1",
           f"--master-port={29541 + world}", bench, "--gpus", str(world), *args]
    r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    out = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in out
    total = rows * world
    assert out["n_gpus"] == world and out["scaling"] == "weak"
    assert out["config"]["parallelism"] == f"dp{world}" and out["config"]["global_batch"] == total
    assert out["value"] == pytest.approx(total / (out["ms_per_step"] / 1e3), rel=1e-6)
    one = subprocess.run([sys.executable, bench, "--rows", str(total), *args[2:]],
                         capture_output=True, text=True, env=env, timeout=600)
    assert one.returncode == 0, one.stderr[-3000:]
    ref = json.loads([l for l in one.stdout.splitlines() if l.startswith("{")][0])
    assert out["ate"] == pytest.approx(ref["ate"], rel=1e-9)
    assert out["se"] == pytest.approx(ref["se"], rel=1e-9)


@pytest.mark.parametrize("world", [2, 4])
def test_gloo_dml_gbdt_bitwise_equals_single(world, tutorial):
    """Config 5's algorithm on real gloo ranks: row-sharded DML-GBDT (global edge sample,
    exact int64 histogram all-reduce per level, exact base and moments) returns the SAME
    BITS as one process at world 2 and 4."""
    script = r"""
import os, sys, json
sys.path.insert(0, %r)
import numpy as np, torch, torch.distributed as dist
dist.init_process_group("gloo")
from ate_replication_causalml_amd.parallel.comm import TorchComm
from ate_replication_causalml_amd.parallel.dist import DistContext
from ate_replication_causalml_amd.data.dgp import make_tutorial_data
from ate_replication_causalml_amd.data.selection import apply_selection_bias
from ate_replication_causalml_amd.estimators.boosting import dml_plr_gbdt
c = TorchComm()
m, _ = apply_selection_bias(make_tutorial_data(6000, 1991))
d = DistContext.for_rank(c, len(m.Y))
r = dml_plr_gbdt(d.local(m.Y), d.local(m.W), d.local(m.X), n_trees=5, depth=3, device="cpu", dist=d)
allv = [None] * c.world_size
dist.all_gather_object(allv, [r.ate.hex(), r.se.hex()])
if c.rank == 0:
    print("RESULT", json.dumps(allv), flush=True)
dist.destroy_process_group()
""" % ROOT
    import json
    import tempfile
    with tempfile.NamedTemporaryFile("w", suffix=".py", delete=False) as f:
        f.write(script)
        path = f.name
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={world}", "--master-addr=127.0.0.1",
           f"--master-port={29561 + world}", path]
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=300)
    finally:
        os.unlink(path)
    assert r.returncode == 0, r.stderr[-3000:]
    got = json.loads([l for l in r.stdout.splitlines() if l.startswith("RESULT")][0].split(" ", 1)[1])
    assert len(got) == world
    from ate_replication_causalml_amd.estimators.boosting import dml_plr_gbdt
    _, m, _ = tutorial
    ref = dml_plr_gbdt(m.Y, m.W, m.X, n_trees=5, depth=3, device="cpu")
    for a, s in got:                               # every rank, every bit
        assert float.fromhex(a) == ref.ate and float.fromhex(s) == ref.se


def _dml_exact(world, rank, comm, n=1500, p=24, block=64):
    pan = synthetic_panel(n, p=p, folds=5, seed=3, dtype="f64", device="cpu", rank=rank,
                          world=world, align=block)
    res, mom, _ = dml_crossfit_panel(pan, 5, comm=comm, exact=True)
    return res.numpy(), mom.numpy()


@pytest.mark.parametrize("world", [2, 4])
def test_exact_mode_dml_bitwise_world_invariant(world):
    """Exact reduction mode: block-aligned shards, the fold Gram stack
    all-reduced as int64 limbs of per-block partials, exact score moments -> the DML ATE,
    SE and moments are the SAME BITS at world 1, 2 and 4 (rtol=0)."""
    ref, mref = _dml_exact(1, 0, LocalComm())
    outs = run_simulated(world, lambda c: _dml_exact(world, c.rank, c))
    for res, mom in outs:
        np.testing.assert_array_equal(res, ref)
        np.testing.assert_array_equal(mom, mref)
    # the exact mode estimates the same quantity as the default mode (rounding only)
    plain, _ = _dml(1, 0, LocalComm())
    np.testing.assert_allclose(ref, plain, rtol=1e-9)


def test_gloo_exact_mode_dml_bitwise():
    """The same on real gloo processes (world 2 and 4 in one launcher call each)."""
    script = r"""
import os, sys, json
sys.path.insert(0, %r)
import torch, torch.distributed as dist
dist.init_process_group("gloo")
from ate_replication_causalml_amd.parallel.comm import TorchComm
from ate_replication_causalml_amd.data.device_dgp import synthetic_panel
from ate_replication_causalml_amd.estimators.lasso import dml_crossfit_panel
c = TorchComm()
pan = synthetic_panel(1500, p=24, folds=5, seed=3, dtype="f64", device="cpu", rank=c.rank,
                      world=c.world_size, align=64)
res, mom, _ = dml_crossfit_panel(pan, 5, comm=c, exact=True)
allv = [None] * c.world_size
dist.all_gather_object(allv, [float(v).hex() for v in res.tolist()])
if c.rank == 0:
    print("RESULT", json.dumps(allv), flush=True)
dist.destroy_process_group()
""" % ROOT
    import json
    import tempfile
    ref, _ = _dml_exact(1, 0, LocalComm())
    want = [float(v).hex() for v in ref.tolist()]
    with tempfile.NamedTemporaryFile("w", suffix=".py", delete=False) as f:
        f.write(script)
        path = f.name
    try:
        for world in (2, 4):
            env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1")
            cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                   f"--nproc-per-node={world}", "--master-addr=127.0.0.1",
                   f"--master-port={29581 + world}", path]
            r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=300)
            assert r.returncode == 0, r.stderr[-3000:]
            got = json.loads([l for l in r.stdout.splitlines()
                              if l.startswith("RESULT")][0].split(" ", 1)[1])
            assert all(g == want for g in got), (world, got, want)
    finally:
        os.unlink(path)


def test_exact_gram_range_guard():
    """The exact mode's fixed 2^24-scale int64 limbs are exact only while every Gram entry
    stays below 2^38: data that could wrap them is refused instead of silently summed
    (the guard bounds |G_jk| by amax_j * amax_k * n_total)."""
    from ate_replication_causalml_amd.ops.gram import check_exact_range, gram
    pan = synthetic_panel(1500, p=24, folds=5, seed=3, dtype="f64", device="cpu", align=64)
    check_exact_range(pan, n_total=pan.n)                       # tutorial-scale data: fine
    with pytest.raises(ValueError, match="limb range"):
        check_exact_range(pan, n_total=10 ** 12)                # weak scaling to 1e12 rows
    pan.data[3, 7] = 1e5                                        # one large entry
    with pytest.raises(ValueError, match="limb range"):
        gram(pan, exact=True)


def test_gloo_config4_causal_forest_bootstrap_bitwise():
    """Config 4 end to end over real gloo processes: the tree-sharded causal forest
    (nuisance and causal forests, int64 fixed-point C05 sums) and the replicate-sharded
    bootstrap (C07) give the SAME BITS as one process, for the forest outputs, the AIPW
    ATE and the bootstrap SE, at world 2 and 3."""
    script = r"""
import os, sys, json
sys.path.insert(0, %r)
import numpy as np, torch, torch.distributed as dist
dist.init_process_group("gloo")
from ate_replication_causalml_amd.parallel.comm import TorchComm
from ate_replication_causalml_amd.estimators import crossfit as CF
from ate_replication_causalml_amd.models import forest as F
c = TorchComm()
r = np.random.default_rng(4)
n = 1200
X = r.normal(size=(n, 6)); W = (r.uniform(size=n) < 0.4).astype(float)
Y = X[:, 0] + (1 + (X[:, 1] > 0)) * W + 0.3 * r.normal(size=n)
b = CF.causal_forest_bootstrap(Y, W, X, num_trees=24, nuisance_trees=12, B=60, compat="textbook", device="cpu",
                               comm=c, boot_chunk=25)
cf = F.causal_forest(X, Y, W, num_trees=24, nuisance_trees=12, seed=12345, backend="cpu", comm=c)
h = lambda a: __import__("hashlib").sha256(np.ascontiguousarray(a).tobytes()).hexdigest()
out = [float(b.ate).hex(), float(b.se).hex(), h(cf.tau_oob), h(cf.var_oob), h(cf.y_hat)]
allv = [None] * c.world_size
dist.all_gather_object(allv, out)
if c.rank == 0:
    print("RESULT", json.dumps(allv), flush=True)
dist.destroy_process_group()
""" % ROOT
    import hashlib
    import json
    import tempfile
    from ate_replication_causalml_amd.estimators import crossfit as CF
    from ate_replication_causalml_amd.models import forest as F
    r = np.random.default_rng(4)
    n = 1200
    X = r.normal(size=(n, 6))
    W = (r.uniform(size=n) < 0.4).astype(float)
    Y = X[:, 0] + (1 + (X[:, 1] > 0)) * W + 0.3 * r.normal(size=n)
    b = CF.causal_forest_bootstrap(Y, W, X, num_trees=24, nuisance_trees=12, B=60, compat="textbook",
                                   device="cpu", boot_chunk=25)
    cf = F.causal_forest(X, Y, W, num_trees=24, nuisance_trees=12, seed=12345, backend="cpu")
    h = lambda a: hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()  # noqa: E731
    want = [float(b.ate).hex(), float(b.se).hex(), h(cf.tau_oob), h(cf.var_oob), h(cf.y_hat)]
    with tempfile.NamedTemporaryFile("w", suffix=".py", delete=False) as f:
        f.write(script)
        path = f.name
    try:
        for world in (2, 3):
            env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1")
            cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                   f"--nproc-per-node={world}", "--master-addr=127.0.0.1",
                   f"--master-port={29601 + world}", path]
            r2 = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=300)
            assert r2.returncode == 0, r2.stderr[-3000:]
            got = json.loads([l for l in r2.stdout.splitlines()
                              if l.startswith("RESULT")][0].split(" ", 1)[1])
            assert all(g == want for g in got), (world, got, want)
    finally:
        os.unlink(path)


def test_bench_emulated_rank_share():
    """ATE_BENCH_EMULATE_WORLD=W (tools/emulate_ranks.sh): bench.py runs rank 0's share of a
    W-rank job in one process through parallel.comm.EmulatedComm -- the tutorial selection
    is planned alone over W x rows kept rows, rank 0's row shard is generated -- and
    prints one JSON line with the world-W global batch."""
    import json
    bench = os.path.join(ROOT, "bench.py")
    env = dict(os.environ, ATE_BENCH_EMULATE_WORLD="3", OMP_NUM_THREADS="1")
    r = subprocess.run([sys.executable, bench, "--rows", "2000", "--p", "24", "--dtype", "f64",
                        "--steps", "1", "--warmup", "1", "--also-rct", "0", "--parity", "0"],
                       capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["config"]["dgp"] == "tutorial"
    assert out["config"]["n_kept"] == 6000 and out["config"]["n_generated"] > 6000
    assert np.isfinite(out["ate"]) and out["value"] > 0


def test_default_backend_one_rank_per_gpu(monkeypatch):
    """RCCL refuses two ranks on one GPU ("Duplicate GPU detected", profiles/r05_rccl):
    more local ranks than GPUs selects gloo, one rank per GPU keeps RCCL."""
    from ate_replication_causalml_amd.parallel import comm as C
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    monkeypatch.setenv("LOCAL_RANK", "1")
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "2")
    assert C.default_backend() == "gloo"
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 8)
    assert C.default_backend() == "nccl"
    monkeypatch.setattr(torch.cuda, "is_available", lambda: False)
    assert C.default_backend() == "gloo"


def test_allreduce_sym_matches_full_allreduce():
    """C01 moves only the upper triangles of the symmetric fold Grams; the result equals a
    full all-reduce of symmetric inputs and is exactly symmetric."""
    from ate_replication_causalml_amd.estimators.lasso import allreduce_sym_
    P, nseg, world = 7, 3, 3

    def stack(r):
        g = torch.Generator().manual_seed(r)
        a = torch.randn(nseg, P, P, dtype=torch.float64, generator=g)
        return a + a.transpose(1, 2)

    def body(c):
        t = stack(c.rank)
        full = t.clone()
        c.all_reduce_(full)
        allreduce_sym_(c, t)
        return t, full
    for t, full in run_simulated(world, body):
        assert torch.equal(t, t.transpose(1, 2))
        assert torch.allclose(t, full, rtol=0, atol=1e-12)
