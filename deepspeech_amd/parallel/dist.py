"""Process-group setup for one-process-per-GPU data parallelism.

The reference is single-process (src/deepSpeech_train.py:425 pins everything to /cpu;
its multi-tower ``average_gradients`` at :193-228 is dead code). Here each rank drives
one MI355X; ``torch.distributed`` with backend "nccl" is RCCL over xGMI on ROCm, "gloo"
is used for CPU tests. Rendezvous is env:// (torchrun sets RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_ADDR / MASTER_PORT).
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist


@dataclass
class DistContext:
    rank: int = 0
    local_rank: int = 0
    world_size: int = 1
    backend: Optional[str] = None
    device: torch.device = torch.device("cpu")

    @property
    def enabled(self) -> bool:
        return self.world_size > 1

    @property
    def is_main(self) -> bool:
        return self.rank == 0

    def barrier(self) -> None:
        if self.enabled:
            if self.backend == "nccl":
                dist.barrier(device_ids=[self.local_rank])
            else:
                dist.barrier()

    def all_reduce_max(self, x: float) -> float:
        if not self.enabled:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=self.device if self.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def all_reduce_sum(self, x: float) -> float:
        if not self.enabled:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=self.device if self.backend == "nccl" else "cpu")
        dist.all_reduce(t)
        return float(t.item())


def init_distributed(device_pref: str = "auto", timeout_s: int = 600, force_group: bool = False) -> DistContext:
    """Initialise from torchrun env vars; a no-op single-process context otherwise.
    force_group: initialise a process group even at world size 1 (RCCL on the GPU), so the
    data-parallel machinery can run and be timed on one device."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_cuda = (device_pref in ("auto", "cuda")) and torch.cuda.is_available()
    if use_cuda:
        # DS2_DEVICE_INDEX pins every rank to one device (multi-rank rehearsal on a 1-GPU box)
        dev_idx = int(os.environ.get("DS2_DEVICE_INDEX", local))
        torch.cuda.set_device(dev_idx)
        device = torch.device("cuda", dev_idx)
    else:
        device = torch.device("cpu")
    ctx = DistContext(rank=rank, local_rank=local, world_size=world, device=device)
    if world > 1 or force_group:
        # RCCL ("nccl") on GPUs; DS2_DIST_BACKEND=gloo runs the same collectives through host
        # memory (ranks sharing one GPU, where RCCL refuses duplicate devices)
        backend = os.environ.get("DS2_DIST_BACKEND") or ("nccl" if use_cuda else "gloo")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if "MASTER_PORT" not in os.environ:          # single process without torchrun
            import socket
            with socket.socket() as sk:
                sk.bind(("127.0.0.1", 0))
                os.environ["MASTER_PORT"] = str(sk.getsockname()[1])
        kw = dict(backend=backend, timeout=datetime.timedelta(seconds=timeout_s), rank=rank, world_size=world)
        if use_cuda and backend == "nccl":
            kw["device_id"] = device
        restart = os.environ.get("TORCHELASTIC_RESTART_COUNT")
        if restart is not None and world > 1 and os.environ.get("TORCHELASTIC_USE_AGENT_STORE") == "True":
            # elastic job (torchrun) whose agent hosts the store for every attempt: every rank
            # is a client of it. Keys of a relaunched attempt live under their own prefix, so
            # no rank can read a peer address left by the killed attempt (observed: gloo
            # connectFullMesh dialling a dead port after a --max-restarts relaunch). Without
            # an agent store nobody would host a client-only store: the default env://
            # rendezvous (rank 0 hosts) is used instead.
            base = dist.TCPStore(os.environ["MASTER_ADDR"], int(os.environ["MASTER_PORT"]), world,
                                 is_master=False, timeout=datetime.timedelta(seconds=timeout_s))
            run_id = os.environ.get("TORCHELASTIC_RUN_ID", "ds2")
            kw["store"] = dist.PrefixStore("ds2/%s/attempt_%s" % (run_id, restart), base)
        if not dist.is_initialized():
            dist.init_process_group(**kw)
        ctx.backend = backend
    return ctx


def shutdown(ctx: DistContext) -> None:
    if ctx.backend is not None and dist.is_initialized():
        dist.destroy_process_group()
