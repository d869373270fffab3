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
import os
import socket

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


class CollectiveError(RuntimeError):
    """A tensor-parallel collective timed out (a peer never arrived): the
    group can no longer agree and must stop."""


ERR_TOKEN = -2            # argmax output of a step whose collectives failed
MAX_TOKEN_ID = (1 << 17) - 1   # token ids carried by the argmax records


def resid_blocks_for(d: int, world: int) -> int:
    """Residual all-reduce workgroups per rank for width ``d`` at TP ``world``
    (also the layout the TP emulation reproduces)."""
    owned = d // world
    for cw in (64, 32, 128, 16, 256, 8):
        nb = owned // cw
        if d % world == 0 and owned % cw == 0 and 1 <= nb <= 64:
            return nb
    raise ValueError(f"no residual all-reduce layout for d = {d}, world = {world}")


class CustomAllReduce:
    # TP decode-step input buffers: up to 128 token rows x 8192 features f32
    DEFAULT_IN_BYTES = 128 * 8192 * 4

    def __init__(self, group=None, slot_bytes: int = 16 << 20, in_bytes: int | None = None,
                 solo: bool = False):
        """``solo``: a one-rank handle with no process group (the single-GPU
        timing of one TP rank's step, ``scripts/config5_projection.py``): every
        collective runs the same kernel over this rank's buffers only."""
        self.group = group
        self.rank = 0 if solo else dist.get_rank(group)
        self.world = 1 if solo else dist.get_world_size(group)
        self.slot_bytes = slot_bytes
        self.in_bytes = self.DEFAULT_IN_BYTES if in_bytes is None else in_bytes
        lib = _lib.kernels()
        self._h = lib.loqa_car_create(self.rank, self.world, slot_bytes, self.in_bytes)
        if not self._h:
            raise RuntimeError("custom all-reduce: staging allocation failed")
        if not solo:
            hs = lib.loqa_car_handle_size()
            buf = ctypes.create_string_buffer(hs)
            _lib.check(lib.loqa_car_handle(self._h, buf), "hipIpcGetMemHandle")
            handles = [None] * self.world
            dist.all_gather_object(handles, bytes(buf.raw), group=group)
            blob = ctypes.create_string_buffer(b"".join(handles), hs * self.world)
            _lib.check(lib.loqa_car_open(self._h, blob), "hipIpcOpenMemHandle")
        # ranks sharing ONE physical GPU (the multi-rank rehearsal on a one-GPU
        # box): kernels that wait on peers must then leave CU slots for them
        ident = (socket.gethostname(), os.environ.get("HIP_VISIBLE_DEVICES",
                                                      os.environ.get("CUDA_VISIBLE_DEVICES", "")),
                 torch.cuda.current_device())
        idents = [ident] if solo else [None] * self.world
        if not solo:
            dist.all_gather_object(idents, ident, group=group)
        self.shared_device = len(set(idents)) < len(idents)
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

    def prologue_wgs(self, d: int) -> int:
        """Grid cap of the decode GEMMs that run this all-reduce (or the
        attention) as their prologue (ops.skinny_fused ``prologue``): 0 (no cap)
        on GPUs of their own; with every rank on one GPU, the ranks' waiting
        grids plus the standalone all-reduce blocks stay well under the 256
        one-workgroup-per-CU slots, so a rank whose items wait on a peer never
        holds the slots that peer needs."""
        env = int(os.environ.get("LOQA_TP_PROLOGUE_WGS", "0"))
        if env > 0 or not self.shared_device:
            return env
        return max(4, (192 - self.world * self.resid_blocks(d)) // self.world)

    def resid_blocks(self, d: int) -> int:
        """Workgroups per rank of ``resid``: each owns a sub-slice of 64
        features (16 f32x4 lanes per row) of this rank's d / world columns, at
        most 64 workgroups; the next norm reads world x blocks statistic tiles."""
        return resid_blocks_for(d, self.world)

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
        rank's masked argmax (-1: nothing allowed). Returns int32 [B]; every
        row is ``ERR_TOKEN`` when a collective of the group timed out."""
        B = idx.numel()
        assert logits.dtype == torch.float32 and logits.stride(-1) == 1 and logits.shape[0] >= B
        assert idx.dtype == torch.int32 and idx.is_contiguous()
        if not self.argmax_fits(lo, logits.shape[1]):
            raise ValueError(f"vocab shard {lo}+{logits.shape[1]} exceeds the argmax records' "
                             f"{MAX_TOKEN_ID + 1} token ids")
        if out is None:
            out = torch.empty(B, dtype=torch.int32, device=idx.device)
        _lib.check(_lib.kernels().loqa_car_argmax(self._h, logits.data_ptr(), logits.stride(0),
                                                  idx.data_ptr(), B, lo, logits.shape[1],
                                                  out.data_ptr(), _lib.stream_ptr(idx)), "car_argmax")
        self.calls += 1
        return out

    @staticmethod
    def argmax_fits(lo: int, shard: int) -> bool:
        return lo >= 0 and shard >= 1 and lo + shard - 1 <= MAX_TOKEN_ID

    def error(self) -> bool:
        v = _lib.kernels().loqa_car_error(self._h)
        if v < 0:
            raise RuntimeError(f"custom all-reduce: error word unreadable (hipError {-v})")
        return bool(v)

    def clear_error(self) -> None:
        _lib.check(_lib.kernels().loqa_car_clear_error(self._h), "car_clear_error")

    # ------------------------------------------------------ start-up check
    def self_test(self, d: int | None = None) -> dict:
        """Run every collective of this group once on seeded random data and
        check it against the host (gloo) reduction of the same data; raise on
        any mismatch, on every rank together (a TP group that
        cannot reduce correctly - a broken IPC mapping, a link, a protocol
        bug - must never start serving).

        * ``__call__``: f32 one-shot and two-shot sizes, bitwise against the
          rank-ordered f32 sum;
        * ``resid``: residual + rank-ordered f32 partial sums, one bf16
          rounding - bitwise; the row statistics within f32 rounding;
        * ``argmax``: the global (max logit, lowest id) over the shards - exact.
        """
        W, r = self.world, self.rank
        dev = self.device
        d = d or 512 * W
        fails: list[str] = []

        def gen(tag: int) -> torch.Generator:
            return torch.Generator().manual_seed(9000 + 131 * tag + r)

        def gather(t: torch.Tensor) -> list[torch.Tensor]:
            parts = [torch.empty_like(t) for _ in range(W)]
            dist.all_gather(parts, t, group=self.group)
            return parts

        calls0 = self.calls
        # 1. in-place all-reduce, one-shot and two-shot
        for n in (4096, 1 << 18):
            x = torch.randn(n, generator=gen(n))
            ref = torch.zeros(n)
            for p in gather(x):
                ref += p
            y = x.to(dev)
            self(y)
            torch.cuda.synchronize(dev)
            if not torch.equal(y.cpu(), ref):
                fails.append(f"all-reduce n={n}: max err {(y.cpu() - ref).abs().max().item():.3g}")
        # 2. the residual epilogue (reduce-scatter + all-gather + statistics)
        Mpad = 16
        nblk = self.resid_blocks(d)
        res0 = torch.randn(Mpad, d, generator=torch.Generator().manual_seed(77)).to(torch.bfloat16)
        part = torch.randn(Mpad, d, generator=gen(1)) * 0.5
        ref = res0.float()
        for p in gather(part):
            ref = ref + p
        ref = ref.to(torch.bfloat16)
        for which in (0, 1):
            pd = part.to(dev)
            _lib.check(_lib.kernels().loqa_car_fill_inbuf(self._h, which, pd.data_ptr(),
                                                          pd.numel() * 4, _lib.stream_ptr(pd)),
                       "car_fill_inbuf")
            resid = res0.to(dev)
            rowsq = torch.zeros(W * nblk * Mpad, dtype=torch.float32, device=dev)
            self.resid(which, resid, rowsq, nblk)
            torch.cuda.synchronize(dev)
            if not torch.equal(resid.cpu(), ref):
                bad = (resid.cpu().float() != ref.float()).sum().item()
                fails.append(f"resid[{which}]: {bad} of {ref.numel()} elements differ")
            sq = rowsq.view(W * nblk, Mpad).sum(0).cpu()
            want = ref.float().square().sum(1)
            if not torch.allclose(sq, want, rtol=1e-5, atol=1e-3):
                fails.append(f"resid[{which}] row statistics: max err {(sq - want).abs().max().item():.3g}")
        # 3. vocab-parallel argmax (self-tagged records)
        B, shard = 8, 1024
        lg = torch.randn(B, shard, generator=gen(2))
        idx = lg.argmax(1).to(torch.int32)
        idx[B - 1] = -1                        # a row with nothing allowed on this shard
        if r == 0:
            idx[B - 2] = -1
        got = self.argmax(lg.to(dev), idx.to(dev), r * shard)
        torch.cuda.synchronize(dev)
        best = [(-float("inf"), -1)] * B
        for q, (l, i) in enumerate(zip(gather(lg), gather(idx))):
            for b in range(B):
                if i[b] >= 0:
                    v, tok = float(l[b, i[b]]), int(i[b]) + q * shard
                    if v > best[b][0] or (v == best[b][0] and tok < best[b][1]):
                        best[b] = (v, tok)
        want = [t for _, t in best]
        if got.cpu().tolist() != want:
            fails.append(f"argmax: {got.cpu().tolist()} != {want}")
        if self.error():
            fails.append("a collective timed out")
        self.calls = calls0
        verdicts = [None] * W
        dist.all_gather_object(verdicts, fails, group=self.group)
        bad = {q: v for q, v in enumerate(verdicts) if v}
        if bad:
            raise CollectiveError(f"custom all-reduce self-test failed: {bad}")
        return {"ranks": W, "checks": 6}

    def close(self) -> None:
        if self._h:
            _lib.kernels().loqa_car_destroy(self._h)
            self._h = None
