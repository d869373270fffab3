"""Behaviour cases of the reference's own suites that the other files do not
re-express:

* arbitration across consecutive utterances and window clearance
  (``collision_detection_test.go:322-459,517-582``);
* the multi-command timing test - five commands of a 50 ms executor, each
  additional command well under 200 ms and the whole queue under N x 200 ms
  (``multi_command_integration_test.go:266-319``, the headline's own test);
* transcription HTTP errors (``stt_client_test.go:344-421``);
* three concurrent progressive-speech sessions and a failing TTS backend
  (``streaming_test.go:365-428``).
"""
import asyncio
import time

import numpy as np
import pytest

from loqa_hub_amd.llm.commands import Command
from loqa_hub_amd.llm.command_queue import CommandQueue
from loqa_hub_amd.llm.http import HTTPResponse, MockHTTPClient
from loqa_hub_amd.llm.stt_client import STTClient
from loqa_hub_amd.llm.tts import TTSResult
from loqa_hub_amd.streaming import Chan
from loqa_hub_amd.streaming.audio_pipeline import StreamingAudioPipeline
from loqa_hub_amd.transport.audio_proto import AudioChunk
from loqa_hub_amd.transport.audio_service import AudioService, RelayStatus, UtteranceResult


class _Proc:
    def __init__(self):
        self.calls = []

    async def process(self, relay_id, request_id, audio, sample_rate):
        self.calls.append(relay_id)
        return UtteranceResult(transcription=f"heard {relay_id}", response_text="ok",
                               intents=["turn_on"], confidence=0.9)


class _Ctx:
    def __init__(self):
        self.sent = []

    async def write(self, msg):
        self.sent.append(msg)


def _pcm(amp, n=1600):
    t = np.arange(n)
    return (amp * np.sin(2 * np.pi * 440 * t / 16000)).astype("<i2").tobytes()


async def _utterance(relay_id, amp, chunks=2):
    yield AudioChunk(relay_id=relay_id, audio_data=_pcm(amp), sample_rate=16000, is_wake_word=True)
    for i in range(chunks):
        await asyncio.sleep(0.005)
        yield AudioChunk(relay_id=relay_id, audio_data=_pcm(amp), sample_rate=16000,
                         is_end_of_speech=(i == chunks - 1))


def test_consecutive_utterances_each_get_a_window():
    """A relay's second utterance, after the first window closed, opens a new
    window and is processed; nothing of the first window is left behind."""
    async def go():
        proc = _Proc()
        svc = AudioService(proc, window_duration=0.03)
        for k in range(3):
            ctx = _Ctx()
            await svc.StreamAudio(_utterance("hall", 6000), ctx)
            assert ctx.sent[-1].success and ctx.sent[-1].transcription == "heard hall"
            assert not svc.is_relay_active("hall")
            assert svc.windows == {} and "hall" not in svc.active_streams
        assert proc.calls == ["hall"] * 3 and svc.stats["windows"] == 3
    asyncio.run(go())


def test_window_clearance_then_new_collision():
    """After a collision the window clears; a new pair of relays arbitrates
    afresh (the earlier loser can win the next window)."""
    async def go():
        proc = _Proc()
        svc = AudioService(proc, window_duration=0.05)
        a, b = _Ctx(), _Ctx()
        await asyncio.gather(svc.StreamAudio(_utterance("a", 9000), a),
                             svc.StreamAudio(_utterance("b", 2000), b))
        assert proc.calls == ["a"]
        assert svc.windows == {}
        a2, b2 = _Ctx(), _Ctx()
        await asyncio.gather(svc.StreamAudio(_utterance("a", 1000), a2),
                             svc.StreamAudio(_utterance("b", 9000), b2))
        assert proc.calls == ["a", "b"]
        assert svc.stats["arbitrations"] == 2 and svc.stats["cancelled"] == 2
    asyncio.run(go())


def test_window_statuses():
    async def go():
        svc = AudioService(_Proc(), window_duration=0.03)
        w = svc.start_arbitration_window("x")
        assert svc.join_arbitration_window("y")
        assert svc.active_streams["x"].status not in (RelayStatus.WINNER, RelayStatus.CANCELLED)
        await asyncio.sleep(0.06)
        st = {svc.active_streams[r].status for r in ("x", "y")}
        assert st == {RelayStatus.WINNER, RelayStatus.CANCELLED} and not w.is_active
    asyncio.run(go())


class _SlowExec:
    def __init__(self, delay):
        self.delay, self.calls = delay, []

    async def execute_command(self, cmd):
        self.calls.append(cmd.entities.get("device"))
        await asyncio.sleep(self.delay)


@pytest.mark.parametrize("n", [1, 3, 5])
def test_each_additional_command_under_200ms(n):
    """multi_command_integration_test.go:266-319: N commands of a 50 ms
    executor; per command well under the 200 ms budget, total < N x 200 ms."""
    cmds = [Command("turn_on", {"device": f"d{i}"}, 0.9, f"on {i}") for i in range(n)]
    ex = _SlowExec(0.05)
    t0 = time.perf_counter()
    r = asyncio.run(CommandQueue(cmds).execute(ex))
    dt = time.perf_counter() - t0
    assert r.success and len(r.completed_items) == n and ex.calls == [f"d{i}" for i in range(n)]
    assert dt < n * 0.2
    per = [i.duration for i in r.completed_items]
    assert all(p < 0.2 for p in per), per


@pytest.mark.parametrize("status", [422, 500])
def test_stt_http_errors(status):
    async def go():
        client = MockHTTPClient({"/health": HTTPResponse(200, b"ok"),
                                 "/v1/audio/transcriptions": HTTPResponse(status, b'{"detail": "x"}')})
        stt = await STTClient.create("http://stt:8000", client=client)
        with pytest.raises(RuntimeError, match=str(status)):
            await stt.transcribe(np.linspace(-1, 1, 1600).astype(np.float32), 16000)
        bad_json = MockHTTPClient({"/health": HTTPResponse(200, b"ok"),
                                   "/v1/audio/transcriptions": HTTPResponse(200, b"not json")})
        stt2 = await STTClient.create("http://stt:8000", client=bad_json)
        with pytest.raises(ValueError):
            await stt2.transcribe(np.linspace(-1, 1, 1600).astype(np.float32), 16000)
        with pytest.raises(ValueError):
            await stt.transcribe(np.ones(16, np.float32), 0)
    asyncio.run(go())


class _TTS:
    def __init__(self, fail_all=False):
        self.fail_all, self.calls = fail_all, []

    async def synthesize(self, text, options=None):
        self.calls.append(text)
        await asyncio.sleep(0.01)
        if self.fail_all:
            raise RuntimeError("tts down")
        return TTSResult(text.encode(), "audio/wav", len(text))

    async def get_available_voices(self):
        return ["v"]

    async def close(self):
        pass


async def _drain(pc):
    out = []
    async for c in pc.audio_chunks:
        out.append(c)
        if c.is_last:
            break
    return out


def test_three_concurrent_sessions_keep_their_order():
    async def go():
        pipe = StreamingAudioPipeline(_TTS(), max_concurrent=2)
        sessions = {}
        for s in ("s1", "s2", "s3"):
            ch = Chan(8)
            sessions[s] = (ch, pipe.start_pipeline(s, ch))
        for s, (ch, _) in sessions.items():
            for i in range(3):
                await ch.put(f"{s} phrase {i}.")
            ch.close()
        got = await asyncio.gather(*[_drain(pc) for _, pc in sessions.values()])
        for s, chunks in zip(sessions, got):
            assert [c.phrase for c in chunks][:3] == [f"{s} phrase {i}." for i in range(3)]
            assert chunks[-1].is_last
        assert sorted(pipe.get_active_pipelines()) == ["s1", "s2", "s3"]
        for s in sessions:
            await pipe.stop_pipeline(s)
        assert pipe.get_active_pipelines() == []
    asyncio.run(go())


def test_failing_tts_still_terminates_the_stream():
    """streaming_test.go:365-391: every synthesis fails - the session still
    ends with its final (is_last) chunk and counts the failures."""
    async def go():
        pipe = StreamingAudioPipeline(_TTS(fail_all=True), max_concurrent=2)
        ch = Chan(4)
        pc = pipe.start_pipeline("f", ch)
        for p in ("one.", "two."):
            await ch.put(p)
        ch.close()
        chunks = await asyncio.wait_for(_drain(pc), 5)
        assert chunks and chunks[-1].is_last
        m = pipe.get_pipeline_metrics("f")
        assert m.failed_synthesis == 2 and m.synthesized_phrases == 0
        await pipe.stop_pipeline("f")
    asyncio.run(go())
