"""Pinned relay-PCM staging (SURVEY §2.4 "Host<->device data path").

Relay audio arrives on the gRPC stream as PCM16-LE chunks. On the GPU path
every chunk is appended, as raw bytes, into a pinned (``hipHostMalloc``) slot
of the native ``PcmStager`` (``csrc/runtime/runtime.cpp``) the moment it
arrives. Two ways to HBM:

* stream-in (the default on GPUs, ``LOQA_PCM_STREAM_IN``): whenever
  ``FLUSH_SAMPLES`` new samples have arrived the stager issues a
  ``hipMemcpyAsync`` of them into the slot's device mirror on the placed H2D
  side stream (``utils/streams.py`` role "h2d"), so the transfer happens while
  the relay is still speaking; at end of speech only the tail crosses PCIe,
  the encoder's stream waits on the slot's last copy event, and a
  device-to-device copy puts the samples in the encoder's batch buffer;
* whole-utterance: one ``hipMemcpyAsync`` at end of speech on the encoder's
  own stream (ordered before the log-mel kernel that reads it).

Utterances longer than one slot (30 s) CHAIN slots (the
reference accumulates relay audio unboundedly, ``audio_service.go:965,1002``):
a full slot is followed by another; with every slot busy the rest is kept on
the host and copied at upload - nothing is dropped below ``MAX_SAMPLES``
(``HUB_MAX_UTTERANCE_S``, default 600 s); past that the overflow is counted
(``overflow_samples``) and logged as an error. Nothing converts the samples on
the host: the reference's per-sample ``bytesToFloat32Array``
(``audio_service.go:1048-1101``) and WAV/HTTP round trip
(``stt_client.go:365-398``) have no counterpart here - the f32 conversion is
the fused ``pcm16_f32_pad`` kernel on the device.

A slot is recycled only after its copy's event has completed (the stager
checks the event on acquire), so a relay can never overwrite samples that are
still in flight.
"""
from __future__ import annotations

import ctypes
import logging
import os
import threading

import numpy as np

from ..ops import _lib

log = logging.getLogger("loqa.pcm")

# samples per stream-in copy (64 KiB: 2 s of 16 kHz PCM16; a 100 ms relay
# chunk is 3.2 KB, so a copy every ~20 chunks)
FLUSH_SAMPLES = int(os.environ.get("LOQA_PCM_FLUSH_SAMPLES", "32768"))
# longest utterance kept (the reference keeps everything; a bound here keeps
# one runaway relay from exhausting host memory)
MAX_SAMPLES = int(float(os.environ.get("HUB_MAX_UTTERANCE_S", "600")) * 16000)


class PCMSlot:
    """One utterance's pinned sample buffer: a chain of stager slots (30 s
    each) plus a host tail when the stager ran out of slots."""

    def __init__(self, stager: "PcmStager", slot: int, stream: bool = True):
        self.stager = stager
        self.stream = stream and stager.stream_in   # copy chunks as they arrive
        self.slots = [slot]
        self.host_tail = bytearray()
        self.released = False
        self._n = 0

    @property
    def slot(self) -> int:
        return self.slots[0]

    def append(self, data: bytes) -> int:
        """Append PCM16-LE bytes (an odd trailing byte is dropped, as the
        reference does); returns the samples kept."""
        n = len(data) & ~1
        room = 2 * (MAX_SAMPLES - self._n)
        if n > room:
            self.stager.note_overflow((n - max(room, 0)) // 2, MAX_SAMPLES)
            n = max(room, 0)
        if n <= 0:
            return 0
        lib = _lib.runtime()
        mv = memoryview(data)[:n]
        kept = 0
        while kept < n:
            if self.host_tail:            # out of pinned slots: the host keeps the rest
                self.host_tail += mv[kept:n]
                kept = n
                break
            cur = self.slots[-1]
            free = 2 * (self.stager.cap - int(lib.loqa_stager_len(self.stager._h, cur)))
            if free <= 0:
                nxt = self.stager.acquire_index()
                if nxt < 0:
                    self.host_tail += mv[kept:n]
                    kept = n
                    break
                self.slots.append(nxt)
                continue
            take = min(free, n - kept)
            got = lib.loqa_stager_append(self.stager._h, cur, bytes(mv[kept:kept + take]), take)
            if got < 0:
                raise RuntimeError("PCM stager slot overflow")
            kept += take
            if self.stream:
                lib.loqa_stager_flush(self.stager._h, cur, FLUSH_SAMPLES)
        self._n += n // 2
        return n // 2

    def __len__(self) -> int:
        return self._n

    def numpy(self) -> np.ndarray:
        """int16 samples: a zero-copy view of the pinned slot when the chain is
        one slot (valid until released), else a host copy of the chain."""
        lib = _lib.runtime()
        parts = []
        for sl in self.slots:
            n = int(lib.loqa_stager_len(self.stager._h, sl))
            p = lib.loqa_stager_host_ptr(self.stager._h, sl)
            parts.append(np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_int16)),
                                               (max(n, 1),))[:n])
        if self.host_tail:
            parts.append(np.frombuffer(bytes(self.host_tail), dtype="<i2"))
        return parts[0] if len(parts) == 1 else np.concatenate(parts)

    def upload(self, dst_ptr: int, max_samples: int, wait_stream: int) -> None:
        """The samples (at most ``max_samples``) to device memory at
        ``dst_ptr``, ordered before the work that follows on ``wait_stream``;
        the slots are released (recycled once their copies complete)."""
        lib = _lib.runtime()
        off = 0
        for sl in self.slots:
            if off >= max_samples:
                break
            n = min(int(lib.loqa_stager_len(self.stager._h, sl)), max_samples - off)
            _lib.check(lib.loqa_stager_upload(self.stager._h, sl, dst_ptr + 2 * off, n,
                                              wait_stream), "stager_upload")
            off += n
        if self.host_tail and off < max_samples:
            import torch
            tail = np.frombuffer(bytes(self.host_tail), dtype="<i2")[: max_samples - off]
            h = torch.from_numpy(tail.copy()).pin_memory()
            self.stager.host_copy(dst_ptr + 2 * off, h, wait_stream)
        self.release()

    def release(self) -> None:
        if not self.released:
            self.released = True
            for sl in self.slots:
                _lib.runtime().loqa_stager_release(self.stager._h, sl)


class PcmStager:
    """Pool of pinned PCM slots (native ``PcmStager``), optionally streaming
    each slot into a device mirror on a caller-placed H2D stream."""

    def __init__(self, nslots: int = 64, cap_samples: int = 480000, own_stream: bool = False,
                 h2d_stream=None):
        self.cap = cap_samples
        self._h = _lib.runtime().loqa_stager_create(nslots, cap_samples, int(own_stream))
        if not self._h:
            raise RuntimeError("PCM stager: pinned allocation failed")
        self._lock = threading.Lock()
        self.overflows = 0
        self.overflow_samples = 0
        self.exhausted = 0
        self.chained = 0
        self.stream_in = False
        self._h2d = h2d_stream
        self._pending: list = []      # (event, pinned host tail) until the copy is done
        if h2d_stream is not None:
            # stream-in needs a device mirror per slot (hipMalloc): on a GPU
            # whose HBM is nearly full (a 70B shard) that can fail - the stager
            # then stays in whole-utterance mode instead of failing every relay
            rc = _lib.runtime().loqa_stager_set_stream(self._h, h2d_stream.cuda_stream, 1)
            if rc == 0:
                self.stream_in = True
            else:
                self._h2d = None
                log.warning("PCM stream-in disabled (device mirrors not allocated, hip error %d): "
                            "whole-utterance uploads", rc)

    def acquire_index(self) -> int:
        with self._lock:
            s = _lib.runtime().loqa_stager_acquire(self._h)
        if s < 0:
            self.exhausted += 1
        return s

    def acquire(self, stream: bool = True) -> PCMSlot | None:
        """A free slot, or None when every slot is busy / in flight.
        ``stream``: copy its samples to HBM as they arrive (stream-in mode)."""
        s = self.acquire_index()
        return None if s < 0 else PCMSlot(self, s, stream)

    def stage(self, samples: np.ndarray) -> PCMSlot | None:
        """A slot (chain) holding a copy of ``samples`` (int16), or None if
        no slot is free. All the samples are here already, so nothing streams:
        the upload is one direct copy on the consuming stream."""
        slot = self.acquire(stream=False)
        if slot is not None:
            slot.append(np.ascontiguousarray(samples, dtype="<i2").tobytes())
            if len(slot.slots) > 1:
                self.chained += 1
        return slot

    def note_overflow(self, samples: int, limit: int) -> None:
        self.overflows += 1
        self.overflow_samples += samples
        log.error("utterance longer than %.0f s: %d samples dropped (HUB_MAX_UTTERANCE_S)",
                  limit / 16000, samples)

    def host_copy(self, dst_ptr: int, pinned, wait_stream: int) -> None:
        """H2D copy of a pinned host tensor (a chain's host tail) ordered on
        ``wait_stream``; the tensor is kept alive until the copy completes."""
        import torch
        self._pending = [(e, t) for e, t in self._pending if not e.query()]
        _lib.check(_lib.runtime().loqa_memcpy_h2d_async(dst_ptr, pinned.data_ptr(),
                                                          pinned.numel() * 2, wait_stream),
                   "memcpy_h2d_async")
        ev = torch.cuda.Event()
        ev.record(torch.cuda.ExternalStream(wait_stream))
        self._pending.append((ev, pinned))

    def close(self) -> None:
        if self._h:
            _lib.runtime().loqa_stager_destroy(self._h)
            self._h = None



class RegisteredPcm:
    """A relay's samples in host memory another process wrote - a slot of the
    DP front end's shared-memory PCM ring (``parallel/dp_serving.py``) that
    this GPU worker pinned with ``hipHostRegister`` - uploaded straight from
    there by ``hipMemcpyAsync`` (no pickled bytes, no staging copy). The
    front end owns the slot and reuses it only after this utterance's result
    came back, so ``release`` has nothing to return."""

    def __init__(self, view: np.ndarray, host_ptr: int):
        self.view, self.host_ptr = view, host_ptr
        self.released = False

    def __len__(self) -> int:
        return int(self.view.size)

    def numpy(self) -> np.ndarray:
        return self.view

    def upload(self, dst_ptr: int, max_samples: int, wait_stream: int) -> None:
        n = min(len(self), max_samples)
        if n > 0:
            _lib.check(_lib.runtime().loqa_memcpy_h2d_async(dst_ptr, self.host_ptr, 2 * n,
                                                              wait_stream), "memcpy_h2d_async")
        self.released = True

    def release(self) -> None:
        self.released = True


def host_register(addr: int, nbytes: int) -> bool:
    """Pin ``nbytes`` of existing host memory at ``addr`` for DMA
    (``hipHostRegister`` on torch's HIP runtime). False if HIP refuses."""
    from ..utils.hip_runtime import hip_runtime
    hip = hip_runtime()
    hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
    hip.hipHostRegister.restype = ctypes.c_int
    return hip.hipHostRegister(ctypes.c_void_p(addr), ctypes.c_size_t(nbytes), 0) == 0


def host_unregister(addr: int) -> None:
    from ..utils.hip_runtime import hip_runtime
    hip = hip_runtime()
    hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
    hip.hipHostUnregister.restype = ctypes.c_int
    hip.hipHostUnregister(ctypes.c_void_p(addr))
