"""RCCL with more ranks than GPUs: each rank of a torch.distributed.run launch takes GPU
LOCAL_RANK % device_count (parallel/comm.local_device), inits the "nccl" (= RCCL) backend
and runs the collectives the estimators use (all-reduce sum/max, all-gather, reduce-scatter,
broadcast), eagerly and inside a captured hipGraph. Rank 0 prints one JSON line.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29511 tools/rccl_probe.py

On a one-GPU box this tells whether RCCL accepts two ranks on one device (NCCL refuses
that as a duplicate GPU); the result is recorded in profiles/.
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from ate_replication_causalml_amd.parallel import comm as C  # noqa: E402


def main():
    t0 = time.time()
    comm = C.from_env()
    r, w = comm.rank, comm.world_size
    dev = torch.device("cuda", C.local_device()) if torch.cuda.is_available() else torch.device("cpu")
    out = {"world": w, "device_count": torch.cuda.device_count(),
           "backend": torch.distributed.get_backend() if w > 1 else "local"}
    x = torch.full((1 << 20,), float(r + 1), dtype=torch.float64, device=dev)
    comm.all_reduce_(x)
    want = w * (w + 1) / 2
    out["all_reduce_ok"] = bool((x == want).all().item())
    m = torch.tensor([float(r)], dtype=torch.float64, device=dev)
    comm.all_reduce_max_(m)
    out["all_reduce_max_ok"] = float(m.item()) == float(w - 1)
    part = torch.full((1024,), r, dtype=torch.int64, device=dev)
    full = torch.empty(1024 * w, dtype=torch.int64, device=dev)
    comm.all_gather_into_(full, part)
    out["all_gather_ok"] = bool((full.view(w, 1024) ==
                                 torch.arange(w, device=dev).view(w, 1)).all().item())
    src = torch.arange(1024 * w, dtype=torch.int64, device=dev)
    mine = torch.empty(1024, dtype=torch.int64, device=dev)
    comm.reduce_scatter_(mine, src)
    out["reduce_scatter_ok"] = bool((mine == w * torch.arange(r * 1024, (r + 1) * 1024,
                                                              device=dev)).all().item())
    comm.barrier()
    if not getattr(comm, "capturable", True):     # gloo: host-staged, not capturable
        out["seconds"] = round(time.time() - t0, 2)
        if r == 0:
            print(json.dumps(out), flush=True)
        torch.distributed.destroy_process_group()
        return
    # captured: the collectives the bench replays inside its graph
    y = torch.full((4096,), float(r + 1), dtype=torch.float32, device=dev)
    s = torch.cuda.Stream(device=dev)
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        comm.all_reduce_(y)                     # warm the communicator outside capture
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    y.fill_(float(r + 1))
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        comm.all_reduce_(y)
    reps = 0
    for _ in range(3):
        y.fill_(float(r + 1))
        g.replay()
        torch.cuda.synchronize()
        reps += int((y == want).all().item())
    out["graph_all_reduce_ok"] = reps == 3
    comm.barrier()
    out["seconds"] = round(time.time() - t0, 2)
    if r == 0:
        print(json.dumps(out), flush=True)
    if w > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
