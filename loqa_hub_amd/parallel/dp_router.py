"""Data-parallel utterance router across the GPUs of one node.

The hub front end (rank 0) owns every relay stream; arbitration winners are
dealt to GPU workers least-loaded-first. In the synchronous batch form used by
the benchmark, rank 0 packs the step's PCM for all ranks into one device
buffer and ``scatter``s it over RCCL/xGMI (one contiguous message per rank -
per-link bound, so few large messages); per-utterance result records are
``all_gather``ed back for the command/metrics plane (D3).

RCCL has no int16 type: PCM16 travels bit-exact as a bfloat16 view.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

from .dist import DistInfo


def pack_pcm(pcms: list[np.ndarray], total_len: int, cap: int = 480000) -> np.ndarray:
    """Concatenate utterances (each truncated to ``cap`` samples) into a
    zero-padded buffer of ``total_len`` samples."""
    out = np.zeros(total_len, np.int16)
    o = 0
    for p in pcms:
        n = min(len(p), cap)
        assert o + n <= total_len, "PCM slot too small"
        out[o:o + n] = p[:n]
        o += n
    return out


def slot_len_for(per_rank: list[list[np.ndarray]], cap: int = 480000) -> int:
    return max(1, max(sum(min(len(p), cap) for p in ps) for ps in per_rank))


def scatter_pcm(info: DistInfo, per_rank: list[list[np.ndarray]] | None, slot_len: int) -> torch.Tensor:
    """Rank 0 passes per-rank PCM lists; every rank receives its packed int16
    samples (concatenated, in utterance order) as a device tensor."""
    if info.world == 1:
        host = torch.from_numpy(pack_pcm(per_rank[0], slot_len))
        return host.to(info.device)
    cdev = info.comm_device
    recv = torch.empty(slot_len, dtype=torch.bfloat16, device=cdev)
    if info.rank == 0:
        packed = np.stack([pack_pcm(p, slot_len) for p in per_rank])
        src = torch.from_numpy(packed)
        if cdev.type == "cuda":
            src = src.pin_memory().to(cdev, non_blocking=True)
        chunks = list(src.view(torch.bfloat16).unbind(0))
        dist.scatter(recv, chunks, src=0)
    else:
        dist.scatter(recv, None, src=0)
    return recv.view(torch.int16).to(info.device)


def gather_records(info: DistInfo, rec: torch.Tensor) -> torch.Tensor:
    """all_gather fixed-shape float64 result records [B, F] -> [world*B, F]."""
    if info.world == 1:
        return rec
    rec = rec.to(info.comm_device)
    out = [torch.empty_like(rec) for _ in range(info.world)]
    dist.all_gather(out, rec)
    return torch.cat(out, 0)


class LeastLoadedRouter:
    """Online routing for the serving path: assign each arbitration winner to
    the GPU worker with the fewest queued utterances (ties -> lowest rank)."""

    def __init__(self, n_workers: int):
        self.load = [0] * n_workers
        self.healthy = [True] * n_workers

    def pick(self) -> int:
        cands = [i for i in range(len(self.load)) if self.healthy[i]]
        if not cands:
            raise RuntimeError("no healthy GPU workers")
        w = min(cands, key=lambda i: (self.load[i], i))
        self.load[w] += 1
        return w

    def done(self, w: int) -> None:
        self.load[w] = max(0, self.load[w] - 1)

    def mark_unhealthy(self, w: int) -> list[int]:
        """Drain a dead worker; returns the ranks still available."""
        self.healthy[w] = False
        self.load[w] = 0
        return [i for i, h in enumerate(self.healthy) if h]
