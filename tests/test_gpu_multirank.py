"""bench.py with two ranks sharing one MI355X (collectives over gloo, host-staged): the
multi-GPU step as the driver runs it -- graph-captured device phases, path solves sharded
over the ranks (plus the in-flight block: three fits on staggered streams) -- gives the ATE/SE of
one process holding all the rows. (RCCL itself: tests/test_gpu_segmented.py.)"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _json(out):
    return json.loads([l for l in out.splitlines() if l.startswith("{")][-1])


def test_two_ranks_on_one_gpu_match_one_process(gpu):
    bench = os.path.join(ROOT, "bench.py")
    args = ["--steps", "3", "--warmup", "1", "--parity", "0", "--also-rct", "0"]
    env = dict(os.environ, ATE_DIST_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node=2", "--master-addr=127.0.0.1", "--master-port=29655",
                        bench, "--gpus", "2", "--rows", "500000", *args],
                       capture_output=True, text=True, env=env, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    two = _json(r.stdout)
    one = subprocess.run([sys.executable, bench, "--rows", "1000000", *args],
                         capture_output=True, text=True, timeout=240)
    assert one.returncode == 0, one.stderr[-3000:]
    ref = _json(one.stdout)
    assert two["hipgraph"] and two["n_gpus"] == 2
    assert two["throughput_inflight"]["inflight"] == 3
    assert two["throughput_inflight"]["fits_agree"]
    # default (non-exact) mode: each rank's Gram chunks hold other rows than the one
    # process's, so the fp32 chunk partials round differently (~1e-9 relative in the ATE);
    # the bitwise world-size comparison is the exact mode's (test below)
    assert two["ate"] == pytest.approx(ref["ate"], rel=1e-7, abs=1e-12)
    assert two["se"] == pytest.approx(ref["se"], rel=1e-7)


@pytest.mark.parametrize("cols,c04,ranks", [(40, "sliced", 2), (37, "sliced", 2),
                                             (40, "allreduce", 2), (40, "sliced", 3)])
def test_cfg5_gbdt_two_ranks_on_one_gpu_bitwise(gpu, cols, c04, ranks):
    """Config 5's row-sharded DML-GBDT (tools/cfg5.py) with two ranks sharing the GPU
    (gloo collectives): device edge sample, per-level int64 histograms reduce-scattered by
    feature slice with the split candidates all-gathered (37 columns: rank 1's slice is one
    feature short) or all-reduced whole (ATE_GBDT_C04=allreduce), exact moments -> the
    SAME BITS as one process holding all rows. Three ranks: slices of 14, 14 and 12
    features."""
    cfg5 = os.path.join(ROOT, "tools", "cfg5.py")
    args = ["--rows", "200000", "--cols", str(cols), "--trees", "6", "--depth", "4"]
    env = dict(os.environ, ATE_DIST_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    if c04 == "allreduce":
        env["ATE_GBDT_C04"] = "allreduce"
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        f"--nproc-per-node={ranks}", "--master-addr=127.0.0.1",
                        "--master-port=29657", cfg5, *args], capture_output=True, text=True,
                       env=env, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    two = _json(r.stdout)
    one = subprocess.run([sys.executable, cfg5, *args], capture_output=True, text=True,
                         timeout=240)
    assert one.returncode == 0, one.stderr[-3000:]
    ref = _json(one.stdout)
    assert two["world"] == ranks and ref["world"] == 1
    assert two["ate_hex"] == ref["ate_hex"] and two["se_hex"] == ref["se_hex"], (two, ref)


def test_exact_mode_two_ranks_on_one_gpu_bitwise(gpu):
    """bench.py --exact (int64-limb Gram all-reduce of block partials, exact moments) with
    two ranks sharing the GPU gives the SAME BITS as one process holding all rows; the
    default mode agrees with exact mode to rounding."""
    bench = os.path.join(ROOT, "bench.py")
    args = ["--steps", "2", "--warmup", "1", "--parity", "0", "--exact", "1", "--also-rct", "0"]
    env = dict(os.environ, ATE_DIST_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node=2", "--master-addr=127.0.0.1", "--master-port=29659",
                        bench, "--gpus", "2", "--rows", "500000", *args],
                       capture_output=True, text=True, env=env, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    two = _json(r.stdout)
    one = subprocess.run([sys.executable, bench, "--rows", "1000000", *args],
                         capture_output=True, text=True, timeout=240)
    assert one.returncode == 0, one.stderr[-3000:]
    ref = _json(one.stdout)
    assert two["exact"] and ref["exact"] and two["n_gpus"] == 2
    assert two["ate_hex"] == ref["ate_hex"] and two["se_hex"] == ref["se_hex"], (two, ref)


def test_cfg3_rf_two_ranks_on_one_gpu_bitwise(gpu):
    """Config 3's tree-parallel RF cross-fit (tools/cfg3.py) with two ranks sharing the GPU
    (gloo collectives): each rank grows its half of the 15 forests side by side, the local
    vote sums are all-reduced once -> the SAME BITS as one process growing every tree."""
    cfg3 = os.path.join(ROOT, "tools", "cfg3.py")
    args = ["--rows", "300000", "--cols", "40", "--trees", "8"]
    env = dict(os.environ, ATE_DIST_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node=2", "--master-addr=127.0.0.1", "--master-port=29661",
                        cfg3, *args], capture_output=True, text=True, env=env, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    two = _json(r.stdout)
    one = subprocess.run([sys.executable, cfg3, *args], capture_output=True, text=True,
                         timeout=240)
    assert one.returncode == 0, one.stderr[-3000:]
    ref = _json(one.stdout)
    assert two["world"] == 2 and ref["world"] == 1 and two["trees_this_rank"] == 4
    assert two["ate_hex"] == ref["ate_hex"] and two["se_hex"] == ref["se_hex"], (two, ref)


def test_cfg4_causal_forest_two_ranks_on_one_gpu_bitwise(gpu):
    """Config 4 (tools/cfg4.py) with two ranks sharing the GPU (gloo collectives): each rank
    grows its little bags of the three forests (C05 int64 sums) and evaluates its half of
    the bootstrap replicates (C07) -> the ATE and the bootstrap SE are the SAME BITS as one
    process growing every tree and evaluating every replicate."""
    cfg4 = os.path.join(ROOT, "tools", "cfg4.py")
    args = ["--rows", "6000", "--trees", "64", "--boot", "100", "--warm", "0", "--compat", "textbook"]
    env = dict(os.environ, ATE_DIST_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node=2", "--master-addr=127.0.0.1", "--master-port=29663",
                        cfg4, *args], capture_output=True, text=True, env=env, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    two = _json(r.stdout)
    one = subprocess.run([sys.executable, cfg4, *args], capture_output=True, text=True,
                         timeout=240)
    assert one.returncode == 0, one.stderr[-3000:]
    ref = _json(one.stdout)
    assert two["world"] == 2 and ref["world"] == 1 and two["causal_trees_this_rank"] == 32
    assert two["ate_hex"] == ref["ate_hex"] and two["se_hex"] == ref["se_hex"], (two, ref)
