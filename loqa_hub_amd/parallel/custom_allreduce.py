"""Custom one-shot all-reduce over IPC-mapped peer buffers.

``CustomAllReduce(group)`` exports each rank's uncached staging region with
``hipIpcGetMemHandle``, exchanges the handles over the process group, opens
the peers' regions and then all-reduces bf16 tensors with one kernel
(``custom_allreduce.hip``): stage -> signal -> read every peer's slice directly
over xGMI -> sum in f32 in a fixed rank order (bitwise identical results on
every rank) -> end barrier. Tensors larger than the staging slot, non-bf16
tensors or sizes not a multiple of 16 bytes fall back to RCCL
(``dist.all_reduce``), which also stays the correctness oracle. f32 tensors
(the decode path all-reduces the o / down projection's split-K slab before its
fused consumer) are summed in f32.

Use as ``TPGroup(rank, world, group, allreduce=CustomAllReduce(group))``.
"""
from __future__ import annotations

import ctypes

import torch
import torch.distributed as dist

from ..ops import _lib


class CustomAllReduce:
    def __init__(self, group=None, slot_bytes: int = 8 << 20):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.slot_bytes = slot_bytes
        lib = _lib.kernels()
        self._h = lib.loqa_car_create(self.rank, self.world, slot_bytes)
        if not self._h:
            raise RuntimeError("custom all-reduce: staging allocation failed")
        hs = lib.loqa_car_handle_size()
        buf = ctypes.create_string_buffer(hs)
        _lib.check(lib.loqa_car_handle(self._h, buf), "hipIpcGetMemHandle")
        handles = [None] * self.world
        dist.all_gather_object(handles, bytes(buf.raw), group=group)
        blob = ctypes.create_string_buffer(b"".join(handles), hs * self.world)
        _lib.check(lib.loqa_car_open(self._h, blob), "hipIpcOpenMemHandle")
        self.calls = 0
        self.fallbacks = 0

    def eligible(self, x: torch.Tensor) -> bool:
        nb = x.numel() * x.element_size()
        return (x.is_cuda and x.dtype in (torch.bfloat16, torch.float32) and x.is_contiguous()
                and nb % 16 == 0 and nb <= self.slot_bytes)

    def __call__(self, x: torch.Tensor) -> torch.Tensor:
        """In-place all-reduce (sum) of ``x``."""
        if self.world == 1:
            return x
        if not self.eligible(x):
            self.fallbacks += 1
            dist.all_reduce(x, group=self.group)
            return x
        _lib.check(_lib.kernels().loqa_car_allreduce(self._h, x.data_ptr(), x.data_ptr(),
                                                     x.numel(), int(x.dtype == torch.float32),
                                                     _lib.stream_ptr(x)),
                   "custom_allreduce")
        self.calls += 1
        return x

    def error(self) -> bool:
        return bool(_lib.kernels().loqa_car_error(self._h))

    def close(self) -> None:
        if self._h:
            _lib.kernels().loqa_car_destroy(self._h)
            self._h = None
