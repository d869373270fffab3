"""Pinned relay-PCM staging (SURVEY §2.4 "Host<->device data path").

Relay audio arrives on the gRPC stream as PCM16-LE chunks. On the GPU path
every chunk is appended, as raw bytes, into a pinned (``hipHostMalloc``) slot
of the native ``PcmStager`` (``csrc/runtime/runtime.cpp``) the moment it
arrives; at end of speech the STT engine moves the slot to HBM with one
``hipMemcpyAsync`` issued on the encoder's own stream (ordered before the
log-mel kernel that reads it). A dedicated H2D stream (the native stager's
``own_stream`` mode) measured 2-4% slower end to end (18.75 / 18.35 vs 19.11 /
19.11 utt/s, docs/PERF.md "Round 4"): created after the serving streams it
lands on an arbitrary hardware queue, and the copy needs the encoder's order
anyway. Nothing converts the samples on the host: the
reference's per-sample ``bytesToFloat32Array`` (``audio_service.go:1048-1101``)
and WAV/HTTP round trip (``stt_client.go:365-398``) have no counterpart here -
the f32 conversion is the fused ``pcm16_f32_pad`` kernel on the device.

A slot is recycled only after its copy's event has completed (the stager
checks the event on acquire), so a relay can never overwrite samples that are
still in flight.
"""
from __future__ import annotations

import ctypes
import threading

import numpy as np

from ..ops import _lib


class PCMSlot:
    """One utterance's pinned sample buffer (a stager slot)."""

    def __init__(self, stager: "PcmStager", slot: int):
        self.stager, self.slot = stager, slot
        self.released = False

    def append(self, data: bytes) -> int:
        """Append PCM16-LE bytes (an odd trailing byte is dropped, as the
        reference does); returns the samples appended (truncates at capacity)."""
        n = len(data) & ~1
        room = 2 * (self.stager.cap - len(self))
        if n > room:
            n = room
            self.stager.overflows += 1
        if n <= 0:
            return 0
        got = _lib.runtime().loqa_stager_append(self.stager._h, self.slot, data, n)
        if got < 0:
            raise RuntimeError("PCM stager slot overflow")
        return got

    def __len__(self) -> int:
        return int(_lib.runtime().loqa_stager_len(self.stager._h, self.slot))

    def numpy(self) -> np.ndarray:
        """Zero-copy int16 view of the pinned samples (valid until released)."""
        n = len(self)
        p = _lib.runtime().loqa_stager_host_ptr(self.stager._h, self.slot)
        return np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_int16)), (max(n, 1),))[:n]

    def upload(self, dst_ptr: int, max_samples: int, wait_stream: int) -> None:
        """hipMemcpyAsync of the samples to ``dst_ptr``, ordered before the
        work that follows on ``wait_stream``. The slot is released (recycled
        once the copy completes)."""
        _lib.check(_lib.runtime().loqa_stager_upload(self.stager._h, self.slot, dst_ptr,
                                                     max_samples, wait_stream), "stager_upload")
        self.release()

    def release(self) -> None:
        if not self.released:
            self.released = True
            _lib.runtime().loqa_stager_release(self.stager._h, self.slot)


class PcmStager:
    """Pool of pinned PCM slots with an H2D stream (native ``PcmStager``)."""

    def __init__(self, nslots: int = 64, cap_samples: int = 480000, own_stream: bool = False):
        self.cap = cap_samples
        self._h = _lib.runtime().loqa_stager_create(nslots, cap_samples, int(own_stream))
        if not self._h:
            raise RuntimeError("PCM stager: pinned allocation failed")
        self._lock = threading.Lock()
        self.overflows = 0
        self.exhausted = 0

    def acquire(self) -> PCMSlot | None:
        """A free slot, or None when every slot is busy / in flight."""
        with self._lock:
            s = _lib.runtime().loqa_stager_acquire(self._h)
        if s < 0:
            self.exhausted += 1
            return None
        return PCMSlot(self, s)

    def stage(self, samples: np.ndarray) -> PCMSlot | None:
        """A slot holding a copy of ``samples`` (int16), or None if none is free."""
        slot = self.acquire()
        if slot is not None:
            slot.append(np.ascontiguousarray(samples, dtype="<i2")[: self.cap].tobytes())
        return slot

    def close(self) -> None:
        if self._h:
            _lib.runtime().loqa_stager_destroy(self._h)
            self._h = None
