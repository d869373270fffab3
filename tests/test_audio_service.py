"""gRPC audio service (C12/C37): PCM conversion, multi-relay wake-word arbitration
(reference ``collision_detection_test.go`` / ``audio_service_test.go``), scoped
windows, and a real grpc.aio round trip."""
import asyncio

import numpy as np
import pytest

from loqa_hub_amd.transport.audio_proto import (AudioChunk, AudioResponse, add_audio_service,
                                                stream_audio_stub)
from loqa_hub_amd.transport.audio_service import (MSG_CANCELLED, AudioService, RelayStatus,
                                                  UtteranceResult, bytes_to_float32_array,
                                                  calculate_signal_strength)


class FakeProcessor:
    def __init__(self):
        self.calls = []

    async def process(self, relay_id, request_id, audio, sample_rate):
        self.calls.append((relay_id, audio.size))
        return UtteranceResult(transcription=f"heard {relay_id}", response_text="ok",
                               intents=["turn_on"], confidence=0.9)


class FakeContext:
    def __init__(self):
        self.sent = []

    async def write(self, msg):
        self.sent.append(msg)


def pcm(amplitude, n=1600):
    t = np.arange(n)
    return (amplitude * np.sin(2 * np.pi * 440 * t / 16000)).astype("<i2").tobytes()


async def relay_stream(relay_id, amp, speech_chunks=3, delay=0.0):
    await asyncio.sleep(delay)
    yield AudioChunk(relay_id=relay_id, audio_data=pcm(amp), sample_rate=16000, is_wake_word=True)
    for i in range(speech_chunks):
        await asyncio.sleep(0.01)
        yield AudioChunk(relay_id=relay_id, audio_data=pcm(amp), sample_rate=16000,
                         is_end_of_speech=(i == speech_chunks - 1))


def test_pcm_conversion_and_rms():
    assert bytes_to_float32_array(b"").size == 0
    a = bytes_to_float32_array(np.array([32767, -32767, 0], "<i2").tobytes() + b"\x01")
    assert np.allclose(a, [1.0, -1.0, 0.0])
    assert calculate_signal_strength(np.zeros(0, np.float32)) == 0.0
    assert calculate_signal_strength(np.full(4, 0.5, np.float32)) == pytest.approx(0.5)


def test_single_relay_processed():
    async def go():
        proc = FakeProcessor()
        svc = AudioService(proc, window_duration=0.05)
        ctx = FakeContext()
        await svc.StreamAudio(relay_stream("kitchen", 8000), ctx)
        assert proc.calls and proc.calls[0][0] == "kitchen"
        assert ctx.sent[-1].transcription == "heard kitchen" and ctx.sent[-1].success
        assert not svc.is_relay_active("kitchen")
    asyncio.run(go())


def test_collision_loudest_relay_wins():
    async def go():
        proc = FakeProcessor()
        svc = AudioService(proc, window_duration=0.1)
        ctxs = {r: FakeContext() for r in ("a", "b", "c")}
        amps = {"a": 2000, "b": 12000, "c": 5000}
        await asyncio.gather(*[svc.StreamAudio(relay_stream(r, amps[r], delay=0.01 * i), ctxs[r])
                               for i, r in enumerate(ctxs)])
        assert [c[0] for c in proc.calls] == ["b"]
        for r in ("a", "c"):
            assert any(m.command == "relay_cancelled" and m.response_text == MSG_CANCELLED
                       for m in ctxs[r].sent)
        assert ctxs["b"].sent[-1].transcription == "heard b"
        assert svc.stats["arbitrations"] == 1 and svc.stats["cancelled"] == 2
    asyncio.run(go())


def test_late_relay_rejected():
    async def go():
        svc = AudioService(FakeProcessor(), window_duration=0.05)
        w = svc.start_arbitration_window("a")
        assert svc.join_arbitration_window("b")
        await asyncio.sleep(0.08)
        assert not w.is_active and w.winner_id in ("a", "b")
        assert not svc.join_arbitration_window("c")
        assert svc.active_streams["a"].status in (RelayStatus.WINNER, RelayStatus.CANCELLED)
    asyncio.run(go())


def test_group_scope_processes_rooms_independently():
    async def go():
        proc = FakeProcessor()
        svc = AudioService(proc, window_duration=0.05, scope="per_relay_group",
                           relay_groups={"k1": "kitchen", "k2": "kitchen", "b1": "bedroom"})
        ctxs = {r: FakeContext() for r in ("k1", "k2", "b1")}
        amps = {"k1": 3000, "k2": 9000, "b1": 1000}
        await asyncio.gather(*[svc.StreamAudio(relay_stream(r, amps[r]), ctxs[r]) for r in ctxs])
        assert sorted(c[0] for c in proc.calls) == ["b1", "k2"]
        assert any(m.command == "relay_cancelled" for m in ctxs["k1"].sent)
    asyncio.run(go())


def test_grpc_roundtrip():
    grpc = pytest.importorskip("grpc")

    async def go():
        server = grpc.aio.server()
        proc = FakeProcessor()
        add_audio_service(server, AudioService(proc, window_duration=0.05))
        port = server.add_insecure_port("127.0.0.1:0")
        await server.start()
        try:
            async with grpc.aio.insecure_channel(f"127.0.0.1:{port}") as ch:
                call = stream_audio_stub(ch)(relay_stream("relay-x", 6000))
                got = [r async for r in call]
            assert got and isinstance(got[-1], AudioResponse)
            assert got[-1].transcription == "heard relay-x" and got[-1].success
        finally:
            await server.stop(0)
    asyncio.run(go())


def test_single_relay_group_bypasses_window():
    """ARBITRATION_SINGLE_RELAY_BYPASS (reference docs/COLLISION_DETECTION.md:203,
    "Single relay: No additional latency"): in the per-group scope a relay
    whose static group has no other member wins at once, while a relay that
    shares its room still waits out the window and collides as before."""
    import time

    async def go():
        proc = FakeProcessor()
        svc = AudioService(proc, window_duration=0.5, scope="per_relay_group",
                           relay_groups={"k1": "kitchen", "k2": "kitchen", "b1": "bedroom"},
                           single_relay_bypass=True)
        assert not svc.can_collide("b1") and not svc.can_collide("garage-relay")
        assert svc.can_collide("k1") and svc.can_collide("k2")
        t0 = time.monotonic()
        ctx_b = FakeContext()
        await svc.StreamAudio(relay_stream("b1", 3000, speech_chunks=2), ctx_b)
        t_single = time.monotonic() - t0
        t0 = time.monotonic()
        ck1, ck2 = FakeContext(), FakeContext()
        await asyncio.gather(svc.StreamAudio(relay_stream("k1", 2000), ck1),
                             svc.StreamAudio(relay_stream("k2", 8000, delay=0.02), ck2))
        t_pair = time.monotonic() - t0
        return proc, svc, ctx_b, ck1, ck2, t_single, t_pair
    proc, svc, ctx_b, ck1, ck2, t_single, t_pair = asyncio.run(go())
    assert ctx_b.sent and ctx_b.sent[-1].success and t_single < 0.3, t_single
    assert svc.stats["bypassed"] == 1
    assert t_pair >= 0.5                       # the kitchen pair waited out the window
    assert ck1.sent[-1].response_text == MSG_CANCELLED and ck2.sent[-1].success
    # without the opt-in the single relay waits for the window as the reference does
    async def ref():
        svc2 = AudioService(FakeProcessor(), window_duration=0.3, scope="per_relay_group",
                            relay_groups={"b1": "bedroom"})
        t0 = time.monotonic()
        await svc2.StreamAudio(relay_stream("b1", 3000, speech_chunks=1), FakeContext())
        return time.monotonic() - t0
    assert asyncio.run(ref()) >= 0.3
