"""Process-group bootstrap: one process per GPU, ``torch.distributed`` over
RCCL (backend "nccl" on ROCm) across the xGMI mesh, gloo on CPU.

Reads RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT (torchrun).
"""
from __future__ import annotations

import logging
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


log = logging.getLogger("loqa.dist")


@dataclass
class DistInfo:
    rank: int = 0
    local_rank: int = 0
    world: int = 1
    device: torch.device = torch.device("cpu")
    backend: str = "none"

    @property
    def is_main(self) -> bool:
        return self.rank == 0

    @property
    def comm_device(self) -> torch.device:
        """Device of the tensors handed to collectives: the GPU under RCCL,
        the host under gloo (CPU runs and the shared-GPU rehearsal)."""
        return self.device if self.backend == "nccl" else torch.device("cpu")


def init_distributed(prefer_gpu: bool = True) -> DistInfo:
    """LOQA_DIST_SHARE_GPU=1 is a rehearsal mode for a one-GPU box: every rank
    runs on cuda:0 and the collectives go over gloo on host tensors (RCCL
    refuses two ranks on one device), so a multi-rank bench exercises the
    per-rank GPU pipelines, the node's broker and the record gathering."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    share = os.environ.get("LOQA_DIST_SHARE_GPU", "0") == "1"
    if share:
        local = 0
    use_gpu = prefer_gpu and torch.cuda.is_available()
    if use_gpu:
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    else:
        device = torch.device("cpu")
    backend = "none"
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        backend = "nccl" if use_gpu and not share else "gloo"
        # no device_id: the RCCL communicator (and its streams) is created at
        # the first collective, not here. HIP hands its few hardware queues to
        # streams in first-use order, and which queues the two decoder streams
        # share moves the pipeline between ~11 and ~19 utt/s (docs/PERF.md, "the
        # 1.8x cliff"); a communicator used before the engines' streams would
        # shift every one of them. Callers exchange startup data through the
        # rendezvous store (``store_exchange``) and issue the first collective
        # once the serving streams are in use.
        dist.init_process_group(backend=backend, rank=rank, world_size=world)
    elif dist.is_initialized():
        backend = dist.get_backend()
    return DistInfo(rank, local, world, device, backend)


def store_exchange(info: DistInfo, key: str, value: str | None = None, timeout_s: float = 300.0) -> str:
    """Rank 0 publishes ``value`` under ``key`` in the rendezvous (TCP) store;
    every rank returns it. No GPU collective (see init_distributed)."""
    if info.world == 1:
        return value or ""
    import datetime
    store = dist.distributed_c10d._get_default_store()
    if info.rank == 0:
        store.set(key, value or "")
    store.wait([key], datetime.timedelta(seconds=timeout_s))
    return store.get(key).decode()


def barrier(info: DistInfo) -> None:
    if info.world > 1:
        if info.comm_device.type == "cuda":
            dist.barrier(device_ids=[info.local_rank])
        else:
            dist.barrier()


def max_over_ranks(info: DistInfo, value: float) -> float:
    if info.world == 1:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=info.comm_device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def shutdown(info: DistInfo) -> None:
    if info.world > 1 and dist.is_initialized():
        dist.destroy_process_group()
