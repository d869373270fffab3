"""Paged KV cache: device storage + block pool.

The block pool lives in the native runtime (``csrc/runtime/runtime.cpp``,
``BlockPool``); a Python twin with the same semantics is used only when the
native library is not built (CPU unit tests).
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from ..ops import _lib


class PyBlockPool:
    """Pure-Python twin of the native BlockPool (prefix cache included)."""

    def __init__(self, num_blocks: int, block_size: int):
        self.num_blocks, self.block_size = num_blocks, block_size
        self.ref = [0] * num_blocks
        self.free = list(range(num_blocks))[::-1]
        self.seqs: dict[int, dict] = {}
        self.prefix: dict[tuple, int] = {}
        self.block_key: dict[int, tuple] = {}

    def _take(self) -> int:
        if not self.free:
            for k, b in list(self.prefix.items()):
                if self.ref[b] == 1:
                    del self.prefix[k]
                    del self.block_key[b]
                    self.ref[b] = 1
                    return b
            return -1
        b = self.free.pop()
        self.ref[b] = 1
        return b

    def _release(self, b: int) -> None:
        self.ref[b] -= 1
        if self.ref[b] == 0:
            self.free.append(b)

    def free_blocks(self) -> int:
        return len(self.free) + sum(1 for b in self.prefix.values() if self.ref[b] == 1)

    def add_seq(self, seq_id: int, toks: list[int]) -> int:
        if seq_id in self.seqs:
            return -1
        bs = self.block_size
        blocks, n = [], 0
        key: tuple = ()
        i = 0
        while i + bs < len(toks):
            key = key + tuple(toks[i:i + bs])
            b = self.prefix.get(key)
            if b is None:
                break
            self.ref[b] += 1
            blocks.append(b)
            n += bs
            i += bs
        self.seqs[seq_id] = {"blocks": blocks, "len": n}
        return n

    def append(self, seq_id: int, n: int) -> list[int] | None:
        s = self.seqs[seq_id]
        bs = self.block_size
        out = []
        for i in range(n):
            pos = s["len"] + i
            bi = pos // bs
            if bi >= len(s["blocks"]):
                b = self._take()
                if b < 0:
                    return None
                s["blocks"].append(b)
            out.append(s["blocks"][bi] * bs + pos % bs)
        s["len"] += n
        return out

    def cache_prefix(self, seq_id: int, toks: list[int]) -> None:
        s = self.seqs[seq_id]
        bs = self.block_size
        key: tuple = ()
        for bi, i in enumerate(range(0, len(toks) - bs + 1, bs)):
            if bi >= len(s["blocks"]):
                break
            key = key + tuple(toks[i:i + bs])
            b = s["blocks"][bi]
            if key not in self.prefix and b not in self.block_key:
                self.prefix[key] = b
                self.block_key[b] = key
                self.ref[b] += 1

    def block_table(self, seq_id: int) -> list[int]:
        return list(self.seqs[seq_id]["blocks"])

    def seq_len(self, seq_id: int) -> int:
        return self.seqs[seq_id]["len"]

    def free_seq(self, seq_id: int) -> None:
        for b in self.seqs.pop(seq_id)["blocks"]:
            self._release(b)

    def truncate(self, seq_id: int, new_len: int) -> None:
        s = self.seqs[seq_id]
        if not 0 <= new_len <= s["len"]:
            raise ValueError("truncate beyond the sequence")
        keep = -(-new_len // self.block_size)
        while len(s["blocks"]) > keep:
            self._release(s["blocks"].pop())
        s["len"] = new_len

    def step_meta(self, seq_ids, ns, B_pad, T_pad, max_blocks, positions, slots, cu, ctx, bt,
                  lidx=None) -> int:
        """Same contract as the native ``loqa_pool_step_meta``."""
        if len(seq_ids) > B_pad or sum(ns) > T_pad or (lidx is not None and len(seq_ids) > len(lidx)):
            return -3
        positions[:T_pad] = 0
        slots[:T_pad] = -1
        bt[:B_pad] = 0
        off = 0
        cu[0] = 0
        for i, (sid, n) in enumerate(zip(seq_ids, ns)):
            if sid not in self.seqs:
                return -1
            start = self.seqs[sid]["len"]
            sl = self.append(sid, n)
            if sl is None:
                return -2
            positions[off:off + n] = range(start, start + n)
            slots[off:off + n] = sl
            off += n
            cu[i + 1] = off
            ctx[i] = start + n
            tab = self.seqs[sid]["blocks"]
            if len(tab) > max_blocks:
                return -3
            bt[i, :len(tab)] = tab
            if lidx is not None:
                lidx[i] = off - 1
        cu[len(seq_ids) + 1:B_pad + 1] = off
        ctx[len(seq_ids):B_pad] = 0
        if lidx is not None:
            lidx[len(seq_ids):] = 0
        return 0


class NativeBlockPool:
    def __init__(self, num_blocks: int, block_size: int):
        self.lib = _lib.runtime()
        self.h = self.lib.loqa_pool_create(num_blocks, block_size)
        self.num_blocks, self.block_size = num_blocks, block_size
        self._buf = np.zeros(4096, dtype=np.int32)

    def __del__(self):
        try:
            self.lib.loqa_pool_destroy(self.h)
        except Exception:
            pass

    def free_blocks(self) -> int:
        return self.lib.loqa_pool_free_blocks(self.h)

    @staticmethod
    def _arr(toks) -> np.ndarray:
        return np.ascontiguousarray(np.asarray(toks, dtype=np.int32))

    def add_seq(self, seq_id: int, toks: list[int]) -> int:
        a = self._arr(toks)
        return int(self.lib.loqa_pool_add_seq(self.h, seq_id, a.ctypes.data_as(ctypes.c_void_p), len(a)))

    def append(self, seq_id: int, n: int) -> list[int] | None:
        out = np.empty(max(n, 1), dtype=np.int32)
        rc = self.lib.loqa_pool_append(self.h, seq_id, n, out.ctypes.data_as(ctypes.c_void_p))
        if rc == -2:
            return None
        if rc != 0:
            raise KeyError(seq_id)
        return out[:n].tolist()

    def cache_prefix(self, seq_id: int, toks: list[int]) -> None:
        a = self._arr(toks)
        self.lib.loqa_pool_cache_prefix(self.h, seq_id, a.ctypes.data_as(ctypes.c_void_p), len(a))

    def block_table(self, seq_id: int) -> list[int]:
        n = self.lib.loqa_pool_block_table(self.h, seq_id,
                                           self._buf.ctypes.data_as(ctypes.c_void_p), len(self._buf))
        if n < 0:
            raise KeyError(seq_id)
        return self._buf[:n].tolist()

    def seq_len(self, seq_id: int) -> int:
        return int(self.lib.loqa_pool_seq_len(self.h, seq_id))

    def free_seq(self, seq_id: int) -> None:
        self.lib.loqa_pool_free_seq(self.h, seq_id)

    def truncate(self, seq_id: int, new_len: int) -> None:
        rc = self.lib.loqa_pool_truncate(self.h, seq_id, new_len)
        if rc == -1:
            raise KeyError(seq_id)
        if rc != 0:
            raise ValueError("truncate beyond the sequence")

    def step_meta(self, seq_ids, ns, B_pad, T_pad, max_blocks, positions, slots, cu, ctx, bt,
                  lidx=None) -> int:
        """One call for a whole step's KV metadata (see runtime.cpp); the numpy
        outputs must be C-contiguous int32 (``lidx`` int64)."""
        ids = np.asarray(seq_ids, dtype=np.int64)
        nn = np.asarray(ns, dtype=np.int32)
        vp = ctypes.c_void_p
        for a in (positions, slots, cu, ctx, bt):
            assert a.dtype == np.int32 and a.flags.c_contiguous
        if lidx is not None:
            assert lidx.dtype == np.int64 and lidx.flags.c_contiguous
        assert positions.size >= T_pad and slots.size >= T_pad and cu.size >= B_pad + 1
        assert ctx.size >= B_pad and bt.size >= B_pad * max_blocks
        return int(self.lib.loqa_pool_step_meta(
            self.h, len(ids), ids.ctypes.data_as(vp), nn.ctypes.data_as(vp), B_pad, T_pad,
            max_blocks, positions.ctypes.data_as(vp), slots.ctypes.data_as(vp),
            cu.ctypes.data_as(vp), ctx.ctypes.data_as(vp), bt.ctypes.data_as(vp),
            lidx.ctypes.data_as(vp) if lidx is not None else None,
            len(lidx) if lidx is not None else 0))


def make_block_pool(num_blocks: int, block_size: int, require_native: bool):
    try:
        return NativeBlockPool(num_blocks, block_size)
    except (_lib.NativeLibraryMissing, OSError):
        if require_native:
            raise
        return PyBlockPool(num_blocks, block_size)


class PagedKVCache:
    def __init__(self, n_layers: int, n_kv: int, head_dim: int, num_blocks: int, block_size: int,
                 device, dtype=torch.bfloat16):
        shape = (n_layers, num_blocks, n_kv, block_size, head_dim)
        self.k = torch.zeros(shape, dtype=dtype, device=device)
        self.v = torch.zeros(shape, dtype=dtype, device=device)
        self.block_size = block_size
        self.num_blocks = num_blocks
        self.pool = make_block_pool(num_blocks, block_size,
                                    require_native=torch.device(device).type == "cuda")

    @staticmethod
    def bytes_per_block(n_layers: int, n_kv: int, head_dim: int, block_size: int) -> int:
        return 2 * n_layers * n_kv * block_size * head_dim * 2
