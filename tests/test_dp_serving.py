"""Data-parallel serving: one worker process per device
behind the least-loaded router, crash / hang detection and re-routing, and
FAULT_INJECT-driven failures. Workers run on the CPU here (spawned processes,
same code path as one process per GPU)."""
import asyncio
import time

import numpy as np
import pytest

from loqa_hub_amd.parallel.dp_serving import DPVoiceProcessor
from loqa_hub_amd.transport.audio_service import UtteranceResult


class _EchoProcessor:
    def __init__(self, spec):
        self.rank = spec["rank"]
        self.hang = spec.get("hang_rank") == self.rank
        self.stats = {"utterances": 0}

    async def process(self, relay_id, request_id, audio, sr):
        if self.hang:
            time.sleep(3600)  # a wedged GPU: the worker's loop never comes back
        await asyncio.sleep(0.02)
        self.stats["utterances"] += 1
        return UtteranceResult(transcription=f"w{self.rank}:{request_id}:{len(audio)}",
                               response_text="ok")


def echo_factory(spec, device):
    return _EchoProcessor(spec)


def _run(spec, n_workers, n_req, **kw):
    async def main():
        dp = DPVoiceProcessor(dict(spec, device="cpu", factory=echo_factory, heartbeat_s=0.1),
                              n_workers, **kw)
        await dp.start()
        try:
            audio = np.zeros(1600, np.float32)
            res = await asyncio.wait_for(asyncio.gather(*[
                dp.process(f"relay-{i}", f"req-{i}", audio, 16000) for i in range(n_req)]), 60)
            return res, dp.metrics()
        finally:
            await dp.close()
    return asyncio.run(main())


def test_dp_routes_to_all_workers():
    res, m = _run({}, 2, 8)
    assert all(r.success for r in res)
    owners = {r.transcription.split(":")[0] for r in res}
    assert owners == {"w0", "w1"}
    assert [r.transcription.split(":")[1] for r in res] == [f"req-{i}" for i in range(8)]
    assert m["healthy"] == 2 and not m["failures"]


def test_dp_worker_crash_is_rerouted():
    res, m = _run({"fault_inject": "gpu_kill:1@2"}, 2, 8)
    assert all(r.success for r in res), [r.error for r in res]
    assert all(r.transcription.startswith("w0:") or r.transcription.startswith("w1:") for r in res)
    assert m["healthy"] == 1
    assert m["failures"] and m["failures"][0]["worker"] == 1
    assert "exited" in m["failures"][0]["reason"]


def test_dp_gpu_hang_is_detected():
    res, m = _run({"hang_rank": 0}, 2, 4, watchdog_s=1.0)
    assert all(r.success and r.transcription.startswith("w1:") for r in res)
    assert m["failures"][0]["worker"] == 0


def test_dp_all_workers_dead_fail_cleanly():
    res, m = _run({"fault_inject": "gpu_kill:0@1"}, 1, 3)
    assert all(not r.success and r.command == "error" for r in res)
    assert m["healthy"] == 0


@pytest.mark.parametrize("spec", ["stt_error", "llm_timeout,nats_down", "gpu_kill:3@2%0.5"])
def test_fault_spec_parsing(spec):
    from loqa_hub_amd.utils.faults import FaultInjector
    fi = FaultInjector(spec)
    assert bool(fi)
    with pytest.raises(ValueError):
        FaultInjector("disk_full")


def test_comm_device_follows_backend():
    """Collective tensors live on the GPU only under RCCL; gloo (CPU runs, the
    shared-GPU rehearsal) gets host tensors."""
    import torch

    from loqa_hub_amd.parallel.dist import DistInfo
    gpu = torch.device("cuda", 0)
    assert DistInfo(device=gpu, backend="nccl", world=2).comm_device == gpu
    assert DistInfo(device=gpu, backend="gloo", world=2).comm_device.type == "cpu"
    assert DistInfo().comm_device.type == "cpu"


class _Pcm16Processor:
    """Takes the raw PCM16 (as GPU workers do) and answers with a digest of
    the samples it received."""
    takes_pcm16 = True

    def __init__(self, spec):
        self.rank = spec["rank"]
        self.stats = {}

    async def process(self, relay_id, request_id, audio, sr, transcript_hint=None, pcm16=None,
                      pcm_slot=None):
        import hashlib
        x = pcm_slot.numpy() if pcm_slot is not None else pcm16
        await asyncio.sleep(0.005)
        return UtteranceResult(transcription=hashlib.sha1(np.ascontiguousarray(x).tobytes()).hexdigest(),
                               response_text=str(x.size))


def pcm16_factory(spec, device):
    return _Pcm16Processor(spec)


def test_dp_pcm_shared_memory_ring(monkeypatch):
    """PCM reaches the workers through their shared-memory
    rings (only the slot index crosses the queue), byte-exact; slots are
    recycled when results come back (more utterances than slots); an
    utterance longer than a slot falls back to inline bytes."""
    import hashlib

    from loqa_hub_amd.parallel import dp_serving
    monkeypatch.setattr(dp_serving, "SHM_SLOTS", 3)
    rng = np.random.default_rng(0)
    pcms = [rng.integers(-32768, 32767, n).astype("<i2") for n in
            [1600, 48000, 480000, 16000] * 4 + [480001]]

    async def main():
        dp = DPVoiceProcessor(dict(device="cpu", factory=pcm16_factory, heartbeat_s=0.1), 2)
        await dp.start()
        try:
            assert len(dp._shm) == 2
            res = []
            for k in range(0, len(pcms), 6):          # waves: slots must come back
                res += await asyncio.wait_for(asyncio.gather(*[
                    dp.process(f"relay-{i}", f"req-{i}", np.zeros(0, np.float32), 16000,
                               pcm16=p) for i, p in enumerate(pcms[k:k + 6], k)]), 60)
            return res, dp.stats, [sorted(f) for f in dp._shm_free]
        finally:
            await dp.close()
    res, st, free = asyncio.run(main())
    assert [r.transcription for r in res] == [hashlib.sha1(p.tobytes()).hexdigest() for p in pcms]
    assert st["pcm_shm_sent"] == len(pcms) - 1 and st["pcm_inline_sent"] == 1
    assert free == [[0, 1, 2], [0, 1, 2]]


def test_dp_pcm_rings_fall_back_when_shm_is_short(monkeypatch):
    """a POSIX segment is sparse, so a tmpfs limit surfaces as
    SIGBUS on first touch. The rings are reserved up front: too little free
    /dev/shm, or a failed reservation, means inline PCM (no rings, no leak)."""
    import collections
    import os as _os

    from loqa_hub_amd.parallel import dp_serving as dps
    FakeSt = collections.namedtuple("FakeSt", "f_bavail f_frsize")
    monkeypatch.setattr(dps.os, "statvfs", lambda p: FakeSt(64 << 20 >> 12, 4096))   # 64 MB free
    assert dps.create_pcm_rings(2, 48, dps.SHM_SLOT_BYTES) == []
    monkeypatch.setattr(dps.os, "statvfs", lambda p: FakeSt(1 << 40 >> 12, 4096))
    made = []
    real_fallocate = getattr(_os, "posix_fallocate", None)

    def failing(fd, off, size):
        made.append(fd)
        if len(made) == 2:
            raise OSError(28, "No space left on device")
        if real_fallocate:
            real_fallocate(fd, off, size)
    monkeypatch.setattr(dps.os, "posix_fallocate", failing, raising=False)
    assert dps.create_pcm_rings(3, 2, 4096) == []
    assert len(made) == 2
    monkeypatch.setattr(dps.os, "posix_fallocate", real_fallocate, raising=False)
    rings = dps.create_pcm_rings(2, 2, 4096)
    try:
        assert len(rings) == 2 and all(m.size >= 8192 for m in rings)
    finally:
        for m in rings:
            m.close()
            m.unlink()


def test_pcm_stager_stream_in_failure_degrades(monkeypatch):
    """when the device mirrors of stream-in cannot be allocated
    (HBM nearly full), the stager logs and stays in whole-utterance mode
    instead of raising from its constructor (which failed every relay)."""
    from loqa_hub_amd.engine import pcm_staging

    class FakeRuntime:
        destroyed = 0

        def loqa_stager_create(self, n, cap, own):
            return 1234

        def loqa_stager_set_stream(self, h, stream, on):
            return 2                      # hipErrorOutOfMemory

        def loqa_stager_destroy(self, h):
            FakeRuntime.destroyed += 1

    fake = FakeRuntime()
    monkeypatch.setattr(pcm_staging._lib, "runtime", lambda: fake)

    class Stream:
        cuda_stream = 99
    st = pcm_staging.PcmStager(4, 1600, h2d_stream=Stream())
    assert st.stream_in is False and st._h2d is None
    st.close()
    assert FakeRuntime.destroyed == 1
