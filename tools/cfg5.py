"""BASELINE config 5 (DML-PLR with histogram-GBDT nuisances, N=1e8, p=2000, full panel
resident across 8 x 288 GB HBM) as one rank per GPU.

    python tools/cfg5.py --rows 100000000 --cols 2000 --trees 100            # 1 process: all rows
    torchrun --nproc-per-node 8 tools/cfg5.py --rows 100000000 ...  # rank r: its rows
    python tools/cfg5.py --rows 100000000 --shard 0/8                    # rank 0's share, alone

Each rank generates its slice of every fold directly in HBM (data/device_dgp, rows are a
pure function of (seed, global row)), bins it on the device from the global edge sample and
runs estimators/boosting.dml_plr_gbdt_panel with a DistContext: histograms (C04) and
moments (C06) all-reduced, results bit-identical at every world size. ``--shard r/W``
runs rank r's work of a W-rank job in one process (collectives replaced by identities:
timing of the per-GPU share only; the ATE/SE is not the full-data one). Rank 0 prints one
JSON line (ATE/SE also as float.hex for bitwise comparisons).
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ate_replication_causalml_amd  # noqa: E402,F401  (HIP queue default before torch's init)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=float, default=1e6)
    ap.add_argument("--cols", type=int, default=100)
    ap.add_argument("--trees", type=int, default=100)
    ap.add_argument("--depth", type=int, default=6)
    ap.add_argument("--folds", type=int, default=5)
    ap.add_argument("--seed", type=int, default=13)
    ap.add_argument("--shard", default=None)
    ap.add_argument("--dgp", default="tutorial", choices=["tutorial", "rct", "tutorial-rct"],
                    help="tutorial: the selection-biased df_mod at scale (N = rows kept)")
    ap.add_argument("--checkpoint", default=None, help="directory: per-fold held-out predictions")
    ap.add_argument("--concurrent", action="store_true",
                    help="fit a fold's E[Y|X] and E[W|X] side by side on two streams "
                         "(default: one after the other)")
    a = ap.parse_args()
    import torch
    from ate_replication_causalml_amd.data.device_dgp import synthetic_panel
    from ate_replication_causalml_amd.estimators.boosting import dml_plr_gbdt_panel
    from ate_replication_causalml_amd.parallel import comm as C
    from ate_replication_causalml_amd.parallel.dist import DistContext
    n = int(a.rows)
    if a.shard:
        r, w = (int(v) for v in a.shard.split("/"))
        comm = C.EmulatedComm(r, w)
    else:
        comm = C.from_env()
    rank, world = comm.rank, comm.world_size
    torch.cuda.set_device(C.local_device())
    dev = torch.device("cuda", torch.cuda.current_device())
    t0 = time.perf_counter()
    pan = synthetic_panel(n, p=a.cols, folds=a.folds, seed=a.seed, dtype="bf16", device=dev,
                          rank=rank, world=world, dgp=a.dgp, comm=comm if world > 1 else None)
    torch.cuda.synchronize()
    t_gen = time.perf_counter() - t0
    dist = DistContext(comm, 0, n) if world > 1 or a.shard else None
    ck = None
    if a.checkpoint:
        from ate_replication_causalml_amd.utils.checkpoint import Checkpoint
        ck = Checkpoint(a.checkpoint, {"cfg": 5, "trees": a.trees, "depth": a.depth})
    comm.barrier()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    r = dml_plr_gbdt_panel(pan, n_trees=a.trees, depth=a.depth, dist=dist, checkpoint=ck,
                           data_key=f"synthetic.{n}.{a.cols}.{a.seed}",
                           concurrent=a.concurrent)
    torch.cuda.synchronize()
    comm.barrier()
    secs = time.perf_counter() - t1
    el = torch.tensor([secs], dtype=torch.float64, device=dev)
    comm.all_reduce_max_(el)
    if rank == 0:
        print(json.dumps({
            "config": 5, "estimator": "DML-PLR 5-fold, GBDT nuisances (E[Y|X], E[W|X]), HBM panel",
            "rows_total": n, "rows_this_rank": pan.n, "p": a.cols, "trees": a.trees,
            "depth": a.depth, "world": world, "shard": a.shard, "dgp": a.dgp,
            "rows_generated": int(pan.n_generated), "concurrent": a.concurrent, "seconds": float(el.item()),
            "generate_s": t_gen, "rows_per_s": n / float(el.item()), "ate": r.ate, "se": r.se,
            "ate_hex": float(r.ate).hex(), "se_hex": float(r.se).hex()}), flush=True)
    if world > 1 and not a.shard:
        import torch.distributed as tdist
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
