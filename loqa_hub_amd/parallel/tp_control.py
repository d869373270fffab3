"""Lock-step scheduling of a tensor-parallel LLM engine group.

Every rank of a TP group runs the same ``LLMEngine`` scheduler loop; each
decode step issues the same collectives on every rank, so every rank must take
the same scheduling decisions. Those decisions are a deterministic function of
the request stream - except for WHEN a request arrives relative to the loop's
iterations. The leader (TP rank 0, which owns the hub front end) therefore
publishes, once per scheduler iteration, the requests that arrived for it, and
every follower replays exactly that (``LLMEngine._schedule``). Sampled tokens
need no exchange: the argmax combine (``CustomAllReduce.argmax``) is bitwise
identical on every rank.

Transport: ``csrc/runtime/tp_control.cpp``, a shared-memory ring in /dev/shm
(the ranks of a TP group share one node). A record is the pickled list of new
request batches (prompt token ids + grammar schema), produced and consumed
only by this package's own processes.
"""
from __future__ import annotations

import ctypes
import os
import pickle

from ..ops import _lib


class TPControl:
    NSLOTS = 64
    SLOT_BYTES = 256 << 10

    def __init__(self, rank: int, world: int, tag: str, group=None):
        """Collective over ``group`` (a CPU process group of the TP ranks):
        the leader creates the ring, every follower then maps it."""
        import torch.distributed as dist
        self.rank, self.world = rank, world
        self.name = f"/loqa_tpctl_{tag}".encode()
        lib = _lib.runtime()
        self._buf = None
        if rank == 0:
            self._h = lib.loqa_tpctl_open(self.name, rank, world, self.NSLOTS, self.SLOT_BYTES)
        if world > 1:
            dist.barrier(group=group)
        if rank != 0:
            self._h = lib.loqa_tpctl_open(self.name, rank, world, self.NSLOTS, self.SLOT_BYTES)
        ok = [None] * world
        if world > 1:
            dist.all_gather_object(ok, bool(self._h), group=group)
        else:
            ok = [bool(self._h)]
        if rank == 0 and self._h:
            lib.loqa_tpctl_unlink(self._h)      # every rank has it mapped
        if not all(ok):
            raise RuntimeError(f"TP control ring {self.name!r}: open failed on ranks "
                               f"{[i for i, v in enumerate(ok) if not v]}")
        self._cap = 16 << 20
        self._buf = ctypes.create_string_buffer(self._cap)
        self._beating = False

    # ------------------------------------------------------------ liveness
    def start_heartbeat(self, period_s: float = 0.25) -> None:
        """Stamp this rank's heartbeat word every ``period_s`` from a daemon
        thread (a follower that dies stops beating; one whose GPU hangs keeps
        beating but trips the collectives' bounded waits instead)."""
        import threading
        if self._beating:
            return
        self._beating = True
        lib = _lib.runtime()

        def run():
            import time
            while self._beating and getattr(self, "_h", None):
                lib.loqa_tpctl_beat(self._h)
                time.sleep(period_s)
        lib.loqa_tpctl_beat(self._h)
        self._beat_thread = threading.Thread(target=run, name=f"tpctl-beat-{self.rank}", daemon=True)
        self._beat_thread.start()

    def beat_ages(self) -> list[float]:
        """Seconds since each rank's last heartbeat (-1: never beat)."""
        lib = _lib.runtime()
        out = []
        for r in range(self.world):
            a = lib.loqa_tpctl_beat_age(self._h, r)
            out.append(-1.0 if a < 0 else a / 1e6)
        return out

    def lost_followers(self, max_age_s: float) -> list[int]:
        """Followers that beat once and then stopped for ``max_age_s``."""
        ages = self.beat_ages()
        return [r for r in range(1, self.world) if ages[r] > max_age_s]

    @property
    def leader(self) -> bool:
        return self.rank == 0

    def publish(self, record, stop: bool = False, timeout_s: float = 300.0) -> None:
        """Leader: one scheduler iteration's record (picklable)."""
        data = pickle.dumps(record, protocol=pickle.HIGHEST_PROTOCOL)
        rc = _lib.runtime().loqa_tpctl_publish(self._h, data, len(data), int(stop),
                                               int(timeout_s * 1e6))
        if rc != 0:
            raise RuntimeError(f"TP control publish failed ({rc}): a follower stopped consuming")

    def recv(self, timeout_s: float = -1.0):
        """Follower: (record, stop) of the next iteration; (None, False) on timeout."""
        lib = _lib.runtime()
        stop = ctypes.c_int(0)
        while True:
            n = lib.loqa_tpctl_recv(self._h, self._buf, self._cap, ctypes.byref(stop),
                                    int(timeout_s * 1e6) if timeout_s >= 0 else -1)
            if n == -3:   # consumed but not copied: the ranks can no longer agree
                raise RuntimeError("TP control record larger than the receive buffer")
            if n == -1:
                return None, False
            if n < 0:
                raise RuntimeError(f"TP control receive failed ({n})")
            return pickle.loads(ctypes.string_at(self._buf, n)), bool(stop.value)

    def close(self) -> None:
        self._beating = False
        t = getattr(self, "_beat_thread", None)
        if t is not None:
            t.join(timeout=2.0)
        if getattr(self, "_h", None):
            _lib.runtime().loqa_tpctl_close(self._h)
            self._h = None


def control_tag() -> str:
    """Per-job ring name: the rendezvous port (+ an optional override)."""
    return os.environ.get("LOQA_TPCTL_TAG") or \
        f"{os.environ.get('MASTER_PORT', '0')}_{os.getuid()}"
