"""BASELINE config 3 (AIPW ATE with random-forest nuisances + 5-fold cross-fit, N=1e7,
p=500, 8 x MI355X) as one rank per GPU. Reference ancestor: doubly_robust
(/root/reference/ate_functions.R:149-207), here the cross-fitted textbook AIPW.

    python tools/cfg3.py --rows 10000000 --cols 500 --trees 100          # 1 process: all trees
    torchrun --nproc-per-node 8 tools/cfg3.py --rows 10000000 ...        # rank r: its trees
    python tools/cfg3.py --rows 10000000 --cols 500 --shard 0/8          # rank 0's share, alone

Every rank generates the WHOLE panel in its HBM (data/device_dgp: rows are a pure function
of (seed, global row), 1e7 x 500 bf16 = 10 GB, binned to 5 GB of uint8) and grows its
shard of the trees of all 15 forests (3 nuisances x 5 folds) side by side on streams;
the forests' local held-out vote sums are all-reduced ONCE, packed (C05,
estimators/crossfit.aipw_rf_crossfit_panel). Votes are integers: the ATE / SE are the same
bits at every world size. ``--shard r/W`` runs rank r's work of a W-rank job in one
process (no collective: timing of the per-GPU share; the ATE is that of the shard's trees).
Rank 0 prints one JSON line (ATE / SE also as float.hex for bitwise comparisons).
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
    ap.add_argument("--folds", type=int, default=5)
    ap.add_argument("--seed", type=int, default=11)
    ap.add_argument("--forest-seed", type=int, default=1991)
    ap.add_argument("--shard", default=None)
    ap.add_argument("--dgp", default="tutorial", choices=["tutorial", "rct", "tutorial-rct"],
                    help="tutorial: the selection-biased df_mod at scale (N = rows kept)")
    ap.add_argument("--serial", action="store_true", help="grow the 15 forests one at a time")
    ap.add_argument("--checkpoint", default=None, help="directory: per-rank local vote sums")
    a = ap.parse_args()
    import torch
    from ate_replication_causalml_amd.data.device_dgp import synthetic_panel
    from ate_replication_causalml_amd.estimators.crossfit import aipw_rf_crossfit_panel
    from ate_replication_causalml_amd.parallel import comm as C
    n = int(a.rows)
    shard = tuple(int(v) for v in a.shard.split("/")) if a.shard else None
    comm = C.LocalComm() if shard else C.from_env()
    rank, world = comm.rank, comm.world_size
    torch.cuda.set_device(C.local_device())
    dev = torch.device("cuda", torch.cuda.current_device())
    t0 = time.perf_counter()
    pan = synthetic_panel(n, p=a.cols, folds=a.folds, seed=a.seed, dtype="bf16", device=dev,
                          dgp=a.dgp)
    torch.cuda.synchronize()
    t_gen = time.perf_counter() - t0
    ck = None
    if a.checkpoint:
        from ate_replication_causalml_amd.utils.checkpoint import Checkpoint
        ck = Checkpoint(a.checkpoint, {"cfg": 3, "trees": a.trees})
    comm.barrier()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    r = aipw_rf_crossfit_panel(pan, num_trees=a.trees, seed=a.forest_seed,
                               comm=comm if world > 1 else None, tree_shard=shard,
                               concurrent=not a.serial, checkpoint=ck,
                               data_key=f"synthetic.{n}.{a.cols}.{a.seed}")
    torch.cuda.synchronize()
    comm.barrier()
    secs = time.perf_counter() - t1
    el = torch.tensor([secs], dtype=torch.float64, device=dev)
    comm.all_reduce_max_(el)
    if rank == 0:
        print(json.dumps({
            "config": 3, "estimator": "AIPW 5-fold cross-fit, RF nuisances (e, mu1, mu0), HBM panel",
            "rows": n, "p": a.cols, "trees_per_forest": a.trees,
            "trees_this_rank": r.diagnostics.get("trees_this_device"), "world": world,
            "shard": a.shard, "serial": a.serial, "dgp": a.dgp,
            "rows_generated": int(pan.n_generated), "seconds": float(el.item()),
            "generate_s": t_gen, "rows_per_s": n / float(el.item()), "ate": r.ate, "se": r.se,
            "ate_hex": float(r.ate).hex(), "se_hex": float(r.se).hex()}), flush=True)
    if world > 1:
        import torch.distributed as tdist
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
