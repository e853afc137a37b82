"""Communicator abstraction.

* :class:`TorchComm` — ``torch.distributed``; on MI355X the ``nccl`` backend IS
  RCCL over xGMI (one process per GPU), on CPU the ``gloo`` backend.
  Collectives are enqueued on the current HIP stream (capturable in a graph).
* :class:`ThreadSimComm` — in-process simulator: ranks are threads sharing host
  memory, reductions run in RANK ORDER, so results are deterministic (CPU tests
  of the distributed algorithms without any cluster).
* :class:`LocalComm` — world size 1, no-op.

All DP algorithms in this package reduce *sufficient statistics* (fold Gram
stacks, histogram stacks, score moments, bootstrap partials), so the data itself
never crosses ranks; messages are KB..MB and the design minimises collective
COUNT (one packed buffer per phase), the right trade on point-to-point xGMI.
"""
from __future__ import annotations

import os
import sys
import threading

import torch


class LocalComm:
    rank = 0
    world_size = 1
    capturable = True          # no-op collectives: nothing to keep out of a graph

    def all_reduce_(self, t):
        return t

    def all_reduce_max_(self, t):
        return t

    def all_reduce_min_(self, t):
        return t

    def all_gather(self, t):
        return [t]

    def all_gather_into_(self, out, t):
        out.copy_(t.reshape(out.shape))
        return out

    def reduce_scatter_(self, out, t):
        out.copy_(t.reshape(out.shape))
        return out

    def broadcast_(self, t, src=0):
        return t

    def barrier(self):
        pass

    def dup(self):
        return self


class EmulatedComm(LocalComm):
    """Rank ``rank`` of a ``world``-rank job run ALONE (tools/cfg3.py / cfg4.py --shard r/W):
    every algorithm takes rank r's share of the work (its row / tree / replicate shard),
    and the collectives return shape-correct local data instead of communicating. The
    values are those of the shard, not of the world-W result: a timing of one GPU's share
    of the job, not a way to compute it."""

    emulated = True       # its collectives do not communicate (data/panel_selection plans alone)

    def __init__(self, rank: int, world: int):
        if not 0 <= rank < world:
            raise ValueError(f"rank {rank} outside a world of {world}")
        self.rank, self.world_size = int(rank), int(world)

    def all_gather(self, t):
        return [t.clone() for _ in range(self.world_size)]

    def all_gather_into_(self, out, t):
        out.copy_(t.reshape(-1).repeat(self.world_size).reshape(out.shape))
        return out

    def reduce_scatter_(self, out, t):
        n = out.numel()
        out.copy_(t.reshape(-1)[self.rank * n:(self.rank + 1) * n].reshape(out.shape))
        return out


class TorchComm:
    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world_size = dist.get_world_size(group)
        # RCCL ("nccl") collectives are enqueued on the current HIP stream and can be
        # captured in a hipGraph (utils/graphs); gloo stages through the host (not
        # capturable: estimators run such collectives eagerly between graph segments)
        self.capturable = dist.get_backend(group) == "nccl"

    def all_reduce_(self, t):
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM, group=self.group)
        return t

    def all_reduce_max_(self, t):
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX, group=self.group)
        return t

    def all_reduce_min_(self, t):
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MIN, group=self.group)
        return t

    def all_gather(self, t):
        out = [torch.empty_like(t) for _ in range(self.world_size)]
        self.dist.all_gather(out, t.contiguous(), group=self.group)
        return out

    def _host_staged(self, *ts):
        # gloo's tensor-form reduce-scatter / all-gather are host-side: device tensors are
        # staged through host copies (gloo rehearsals only; RCCL runs them on the device)
        return not self.capturable and any(x.is_cuda for x in ts)

    def all_gather_into_(self, out, t):
        """out (contiguous, world * t.numel() elements) = rank-ordered concatenation."""
        if self._host_staged(out, t):
            h = torch.empty(out.shape, dtype=out.dtype)
            self.dist.all_gather_into_tensor(h, t.cpu().contiguous(), group=self.group)
            return out.copy_(h)
        self.dist.all_gather_into_tensor(out, t.contiguous(), group=self.group)
        return out

    def reduce_scatter_(self, out, t):
        """out = this rank's chunk (rank-ordered, out.numel() elements each) of the SUM of
        every rank's t: (W-1)/W of t's bytes on each ring link, half an all-reduce."""
        if self._host_staged(out, t):
            h = torch.empty(out.shape, dtype=out.dtype)
            self.dist.reduce_scatter_tensor(h, t.cpu().contiguous(), op=self.dist.ReduceOp.SUM,
                                            group=self.group)
            return out.copy_(h)
        self.dist.reduce_scatter_tensor(out, t.contiguous(), op=self.dist.ReduceOp.SUM,
                                        group=self.group)
        return out

    def dup(self):
        """A second communicator over the same ranks (a new process group; a collective
        call: every rank creates it in the same order). Concurrently running fits each need
        their own, so their collectives cannot interleave differently on different ranks."""
        ranks = self.dist.get_process_group_ranks(self.group) if self.group is not None \
            else list(range(self.dist.get_world_size()))
        return TorchComm(self.dist.new_group(ranks))

    def broadcast_(self, t, src=0):
        self.dist.broadcast(t, src=src, group=self.group)
        return t

    def barrier(self):
        if self.dist.get_backend(self.group) == "nccl":
            # RCCL barrier via a tiny all-reduce on the current device (avoids
            # device-guessing warnings)
            x = torch.zeros(1, device=torch.cuda.current_device())
            self.dist.all_reduce(x, group=self.group)
            torch.cuda.synchronize()
        else:
            self.dist.barrier(group=self.group)


class _SimWorld:
    def __init__(self, n):
        self.n = n
        self.barrier = threading.Barrier(n)
        self.slots = [None] * n
        self.lock = threading.Lock()


class ThreadSimComm:
    """Rank ``rank`` of an in-process simulated world (use :func:`run_simulated`)."""

    capturable = False

    def __init__(self, world: _SimWorld, rank: int):
        self.w = world
        self.rank = rank
        self.world_size = world.n

    def _reduce(self, t, op):
        self.w.slots[self.rank] = t.detach().clone()
        self.w.barrier.wait()
        acc = self.w.slots[0].clone()
        for r in range(1, self.world_size):    # fixed rank order -> deterministic
            acc = op(acc, self.w.slots[r])
        self.w.barrier.wait()
        t.copy_(acc)
        return t

    def all_reduce_(self, t):
        return self._reduce(t, lambda a, b: a + b)

    def all_reduce_max_(self, t):
        return self._reduce(t, torch.maximum)

    def all_reduce_min_(self, t):
        return self._reduce(t, torch.minimum)

    def all_gather(self, t):
        self.w.slots[self.rank] = t.detach().clone()
        self.w.barrier.wait()
        out = [s.clone() for s in self.w.slots]
        self.w.barrier.wait()
        return out

    def all_gather_into_(self, out, t):
        parts = self.all_gather(t)
        out.copy_(torch.cat([q.reshape(-1) for q in parts]).reshape(out.shape))
        return out

    def reduce_scatter_(self, out, t):
        acc = self._reduce(t.detach().clone(), lambda a, b: a + b).reshape(-1)
        n = out.numel()
        out.copy_(acc[self.rank * n:(self.rank + 1) * n].reshape(out.shape))
        return out

    def broadcast_(self, t, src=0):
        if self.rank == src:
            self.w.slots[src] = t.detach().clone()
        self.w.barrier.wait()
        t.copy_(self.w.slots[src])
        self.w.barrier.wait()
        return t

    def barrier(self):
        self.w.barrier.wait()


def capturable(comm) -> bool:
    """Whether ``comm``'s collectives may sit inside a captured hipGraph."""
    return comm is None or bool(getattr(comm, "capturable", False))


def run_simulated(world_size: int, fn):
    """Run ``fn(comm)`` on ``world_size`` threads; returns the per-rank results."""
    world = _SimWorld(world_size)
    results = [None] * world_size
    errors = []

    def worker(r):
        try:
            results[r] = fn(ThreadSimComm(world, r))
        except BaseException as e:  # noqa: BLE001
            errors.append(e)
            world.barrier.abort()

    ts = [threading.Thread(target=worker, args=(r,)) for r in range(world_size)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    if errors:
        raise errors[0]
    return results


def local_device() -> int:
    """GPU of this rank: LOCAL_RANK, wrapped over the visible devices (one rank per GPU on
    a full node; ranks share GPUs only when launched with more ranks than devices)."""
    return int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())


def default_backend() -> str:
    """RCCL ("nccl") with one rank per GPU; gloo without a GPU, or when the node runs more
    ranks than it has GPUs: RCCL refuses two ranks on one device at communicator init
    ("Duplicate GPU detected", measured on a one-GPU MI355X box, profiles/r05_rccl)."""
    if not torch.cuda.is_available():
        return "gloo"
    local = int(os.environ.get("LOCAL_WORLD_SIZE", "1"))
    ndev = torch.cuda.device_count()
    if local > ndev:
        if int(os.environ.get("LOCAL_RANK", "0")) == 0:
            print(f"[comm] {local} ranks on {ndev} GPU(s): RCCL needs one rank per GPU, "
                  "using gloo (host-staged collectives)", file=sys.stderr, flush=True)
        return "gloo"
    return "nccl"


def from_env():
    """TorchComm if launched under torch.distributed.run (WORLD_SIZE>1), else LocalComm."""
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        import torch.distributed as dist
        if not dist.is_initialized():
            # ATE_DIST_BACKEND=gloo: host-staged collectives (e.g. several ranks sharing one
            # GPU in a rehearsal); default RCCL ("nccl") when a GPU is visible
            backend = os.environ.get("ATE_DIST_BACKEND") or default_backend()
            # RCCL errors (a failed peer, a timed-out collective) abort the process
            # instead of leaving the other ranks blocked
            os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
            if torch.cuda.is_available():
                torch.cuda.set_device(local_device())
            dist.init_process_group(backend=backend)
        return TorchComm()
    return LocalComm()
