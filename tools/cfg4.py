"""BASELINE config 4 (causal-forest CATE -> ATE with a 1000-replicate bootstrap SE sharded
across 8 x MI355X) as one rank per GPU. Reference: grf::causal_forest + estimate_average_
effect (/root/reference/ate_replication.Rmd:250-265) with the bootstrap of fixed nuisances
of ate_functions.R:188-195 (E10 semantics: the AIPW scores are resampled, no refit).

    python tools/cfg4.py --rows 50000                       # 1 process: all trees, all reps
    torchrun --nproc-per-node 8 tools/cfg4.py --rows 50000  # rank r: its trees and reps
    python tools/cfg4.py --rows 50000 --shard 0/8           # rank 0's share of 8, alone

Data: the tutorial's selection-biased df_mod at n = --rows KEPT rows (data/panel_selection
.selected_rows: calibrated model, ate_replication.Rmd:97-121 over generated-row order).
Every rank holds all rows (the binned / value-rank matrix is replicated) and grows its
shard of the trees of the three forests (Y.hat and W.hat orthogonalisation forests, the
causal forest: whole little bags per rank, C05 int64 fixed-point sums), then evaluates its
B / W bootstrap replicates of mean(Gamma) (C07 all-gather). ``--shard r/W`` runs rank r's
work in one process with no collective (parallel/comm.EmulatedComm: its tree shards, its
replicates; the printed ATE is that of the shard's trees): the per-GPU time of a W-GPU
job. Rank 0 prints one JSON line (ATE / SE also as float.hex).
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
    ap.add_argument("--rows", type=float, default=5e4)
    ap.add_argument("--trees", type=int, default=2000)
    ap.add_argument("--nuisance-trees", type=int, default=None)
    ap.add_argument("--boot", type=int, default=1000)
    ap.add_argument("--seed", type=int, default=1991, help="data / bootstrap seed")
    ap.add_argument("--forest-seed", type=int, default=12345)
    ap.add_argument("--shard", default=None)
    ap.add_argument("--warm", type=int, default=1, help="untimed passes before the timed one")
    ap.add_argument("--compat", default="reference")
    a = ap.parse_args()
    import torch
    from ate_replication_causalml_amd.data.panel_selection import selected_rows
    from ate_replication_causalml_amd.estimators.crossfit import causal_forest_bootstrap
    from ate_replication_causalml_amd.models import forest as F
    from ate_replication_causalml_amd.parallel import comm as C
    n = int(a.rows)
    if a.shard:
        r_, w_ = (int(v) for v in a.shard.split("/"))
        comm = C.EmulatedComm(r_, w_)
    else:
        comm = C.from_env()
    rank, world = comm.rank, comm.world_size
    if torch.cuda.is_available():
        torch.cuda.set_device(C.local_device())
        dev = torch.device("cuda", torch.cuda.current_device())
    else:
        dev = torch.device("cpu")
    t0 = time.perf_counter()
    d, sel = selected_rows(n, a.seed, device=dev)
    t_gen = time.perf_counter() - t0

    def run():
        return causal_forest_bootstrap(d.Y, d.W, d.X, num_trees=a.trees, B=a.boot,
                                       seed=a.forest_seed, boot_seed=a.seed, device=dev,
                                       comm=comm if world > 1 else None,
                                       nuisance_trees=a.nuisance_trees, compat=a.compat)

    for _ in range(a.warm):
        run()

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize()
    sync()
    comm.barrier()
    t1 = time.perf_counter()
    r = run()
    sync()
    comm.barrier()
    secs = time.perf_counter() - t1
    el = torch.tensor([secs], dtype=torch.float64, device=dev)
    comm.all_reduce_max_(el)
    g = 2
    t_first, t_cnt = F.tree_shard(a.trees, g, rank, world)
    from ate_replication_causalml_amd.parallel.dist import shard_range
    if rank == 0 or a.shard:
        print(json.dumps({
            "config": 4, "estimator": "causal forest (grf semantics) + AIPW ATE, "
                                      f"{a.boot}-replicate bootstrap SE",
            "data": "tutorial df_mod (selection-biased), kept rows", "rows": n,
            "rows_generated": sel.n_gen, "trees": a.trees, "boot": a.boot,
            "splits": F.resolve_splits("auto", n), "world": world, "shard": a.shard,
            "emulated": bool(a.shard), "causal_trees_this_rank": t_cnt,
            "boot_reps_this_rank": shard_range(a.boot, rank, world)[1],
            "seconds": float(el.item()), "data_s": t_gen, "ate": r.ate, "se": r.se,
            "se_aipw": r.diagnostics.get("se_aipw"), "ate_hex": float(r.ate).hex(),
            "se_hex": float(r.se).hex()}), flush=True)
    if world > 1 and not a.shard:
        import torch.distributed as tdist
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
