"""Custom all-reduce over IPC-mapped peer buffers.

``CustomAllReduce(group)`` exports each rank's uncached staging region with
``hipIpcGetMemHandle``, exchanges the handles over the (CPU) process group,
opens the peers' regions, and then runs every tensor-parallel collective as ONE
kernel (``csrc/kernels/custom_allreduce.hip``) that reads all peers directly over
the point-to-point xGMI links:

* ``__call__(x)``: in-place sum of a bf16 / f32 tensor - one-shot below 512 KB
  (decode), two-shot reduce-scatter + all-gather above (prefill); tensors
  larger than the staging slot go slot by slot. Host tensors, other dtypes or
  sizes not a multiple of 16 bytes fall back to ``dist.all_reduce``, which
  also stays the correctness oracle.
* ``resid(which, residual, rowsq, ...)``: the TP decode step's row-parallel
  epilogue. The o / down GEMM wrote its f32 partial straight into
  ``inbuf(which)``; the kernel reduce-scatters the partials onto the
  replicated residual stream (f32 sums in a fixed rank order, one bf16
  rounding), all-gathers the rounded slices, and writes the row sums of
  squares the next fused GEMM's RMSNorm prologue reads.
* ``argmax(logits, idx, lo)``: vocab-parallel masked argmax combine - each
  rank's best (logit, token) per row as one self-tagged 64-bit record, max
  over ranks, ties to the lowest token id.

All three are graph-capturable (the call epoch is a device counter).

Use as ``TPGroup(rank, world, group, allreduce=CustomAllReduce(group))``.
"""
from __future__ import annotations

import ctypes

import torch
import torch.distributed as dist

from ..ops import _lib


class DeviceView:
    """A raw device buffer in the shape of a contiguous 2-D tensor, for kernels
    that take (pointer, leading dimension) - the IPC input buffers are not
    torch allocations."""

    def __init__(self, ptr: int, rows: int, cols: int, device: torch.device,
                 dtype: torch.dtype = torch.float32):
        self._ptr, self.shape = ptr, (rows, cols)
        self.dtype, self.device = dtype, device

    def data_ptr(self) -> int:
        return self._ptr

    def stride(self, dim: int = 0) -> int:
        return self.shape[1] if dim == 0 else 1


class CustomAllReduce:
    # TP decode-step input buffers: up to 128 token rows x 8192 features f32
    DEFAULT_IN_BYTES = 128 * 8192 * 4

    def __init__(self, group=None, slot_bytes: int = 16 << 20, in_bytes: int | None = None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.slot_bytes = slot_bytes
        self.in_bytes = self.DEFAULT_IN_BYTES if in_bytes is None else in_bytes
        lib = _lib.kernels()
        self._h = lib.loqa_car_create(self.rank, self.world, slot_bytes, self.in_bytes)
        if not self._h:
            raise RuntimeError("custom all-reduce: staging allocation failed")
        hs = lib.loqa_car_handle_size()
        buf = ctypes.create_string_buffer(hs)
        _lib.check(lib.loqa_car_handle(self._h, buf), "hipIpcGetMemHandle")
        handles = [None] * self.world
        dist.all_gather_object(handles, bytes(buf.raw), group=group)
        blob = ctypes.create_string_buffer(b"".join(handles), hs * self.world)
        _lib.check(lib.loqa_car_open(self._h, blob), "hipIpcOpenMemHandle")
        self.device = torch.device("cuda", torch.cuda.current_device())
        self.calls = 0
        self.fallbacks = 0

    def eligible(self, x: torch.Tensor) -> bool:
        nb = x.numel() * x.element_size()
        return (x.is_cuda and x.dtype in (torch.bfloat16, torch.float32) and x.is_contiguous()
                and nb % 16 == 0)

    def __call__(self, x: torch.Tensor) -> torch.Tensor:
        """In-place all-reduce (sum) of ``x``; tensors larger than the staging
        slot go as consecutive slot-sized calls (long prefill batches)."""
        if self.world == 1:
            return x
        if not self.eligible(x):
            self.fallbacks += 1
            dist.all_reduce(x, group=self.group)
            return x
        flat = x.view(-1)
        es = x.element_size()
        step = (self.slot_bytes // (16 * self.world)) * 16 * self.world // es
        for i in range(0, flat.numel(), step):
            part = flat[i:i + step]
            _lib.check(_lib.kernels().loqa_car_allreduce(self._h, part.data_ptr(), part.data_ptr(),
                                                         part.numel(), int(x.dtype == torch.float32),
                                                         _lib.stream_ptr(x)),
                       "custom_allreduce")
            self.calls += 1
        return x

    # ------------------------------------------------------ TP decode step
    def inbuf(self, which: int, rows: int, cols: int) -> DeviceView:
        """This rank's input buffer ``which`` (0: o projection, 1: down) viewed
        as a [rows, cols] f32 GEMM output."""
        if rows * cols * 4 > self.in_bytes:
            raise ValueError(f"TP input buffer holds {self.in_bytes} bytes, need {rows * cols * 4}")
        p = _lib.kernels().loqa_car_inbuf(self._h, which)
        if not p:
            raise RuntimeError("custom all-reduce: no input buffers")
        return DeviceView(p, rows, cols, self.device)

    def resid_blocks(self, d: int) -> int:
        """Workgroups per rank of ``resid``: each owns a sub-slice of 64
        features (16 f32x4 lanes per row) of this rank's d / world columns, at
        most 64 workgroups; the next norm reads world x blocks statistic tiles."""
        owned = d // self.world
        for cw in (64, 32, 128, 16, 256, 8):
            nb = owned // cw
            if d % self.world == 0 and owned % cw == 0 and 1 <= nb <= 64:
                return nb
        raise ValueError(f"no residual all-reduce layout for d = {d}, world = {self.world}")

    def resid(self, which: int, residual: torch.Tensor, rowsq: torch.Tensor, nblk: int) -> None:
        """residual += sum over ranks of inbuf(which); row sums of squares ->
        rowsq[:world * nblk * Mpad] as world * nblk tiles."""
        Mpad, d = residual.shape
        assert residual.dtype == torch.bfloat16 and residual.is_contiguous()
        assert rowsq.dtype == torch.float32 and rowsq.numel() >= self.world * nblk * Mpad
        _lib.check(_lib.kernels().loqa_car_resid(self._h, which, residual.data_ptr(),
                                                 rowsq.data_ptr(), Mpad, d, nblk,
                                                 _lib.stream_ptr(residual)), "car_resid")
        self.calls += 1

    def argmax(self, logits: torch.Tensor, idx: torch.Tensor, lo: int,
               out: torch.Tensor | None = None) -> torch.Tensor:
        """Global masked argmax over the vocab shards: ``logits`` [B, V/tp] f32
        (this rank's shard, global ids lo..lo+V/tp), ``idx`` [B] int32 this
        rank's masked argmax (-1: nothing allowed). Returns int32 [B]."""
        B = idx.numel()
        assert logits.dtype == torch.float32 and logits.stride(-1) == 1 and logits.shape[0] >= B
        assert idx.dtype == torch.int32 and idx.is_contiguous()
        if out is None:
            out = torch.empty(B, dtype=torch.int32, device=idx.device)
        _lib.check(_lib.kernels().loqa_car_argmax(self._h, logits.data_ptr(), logits.stride(0),
                                                  idx.data_ptr(), B, lo, out.data_ptr(),
                                                  _lib.stream_ptr(idx)), "car_argmax")
        self.calls += 1
        return out

    def error(self) -> bool:
        return bool(_lib.kernels().loqa_car_error(self._h))

    def close(self) -> None:
        if self._h:
            _lib.kernels().loqa_car_destroy(self._h)
            self._h = None
