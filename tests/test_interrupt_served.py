"""A new wake-word winner on a relay interrupts the reply that relay is still
receiving (``streaming_interrupt_handler.go:69-119``, composed into the hub:
VERDICT r3 next-round #6). The progressive reply is a streaming session of the
composed ``StreamingComponents``: registered with the interrupt handler while
it is spoken, recorded (first token / first phrase / completion or interrupt)
in the streaming metrics when it ends."""
import asyncio

import numpy as np

from loqa_hub_amd import config as cfgmod
from loqa_hub_amd.llm.tts import TTSResult
from loqa_hub_amd.server import build_gpu_processor
from loqa_hub_amd.streaming.components import StreamingComponents

HINT = "hey loqa turn on the kitchen lights and then play some jazz"


class SlowTTS:
    """Each phrase takes ``delay`` s: a reply is still being spoken long
    after its decode ended."""

    def __init__(self, delay=0.4):
        self.delay = delay
        self.calls = 0

    async def synthesize(self, text, options=None):
        self.calls += 1
        await asyncio.sleep(self.delay)
        from loqa_hub_amd.engine.tts_engine import pcm16_to_wav
        return TTSResult(pcm16_to_wav(np.zeros(2205, np.int16), 22050), "audio/wav", 4454, 22050)

    async def get_available_voices(self):
        return ["af_bella"]


def _pcm():
    t = np.arange(32000) / 16000.0
    return (6000 * np.sin(2 * np.pi * 220 * t)).astype(np.int16)


def _proc(tts, **env):
    cfg = cfgmod.load({"HUB_STT_MODEL": "test-whisper", "HUB_LLM_MODEL": "test-tiny",
                       "HUB_MAX_BATCH": "4", "STREAMING_ENABLED": "true",
                       "STREAMING_MAX_TOKENS_PER_PHRASE": "2", **env})
    proc = build_gpu_processor(cfg, None, "cpu", tts, bridge=False)
    comps = StreamingComponents.for_processor(cfg, proc)
    proc.attach_streaming(comps)
    return proc, comps


def test_new_winner_interrupts_reply_cpu():
    tts = SlowTTS()
    proc, comps = _proc(tts)

    async def go():
        first = asyncio.ensure_future(proc.process("relay-a", "req-1", None, 16000,
                                                   transcript_hint=HINT, pcm16=_pcm()))
        # wait until relay-a's reply is being spoken
        for _ in range(2000):
            sp = proc._speaking.get("relay-a")
            if sp is not None and sp.t_first_phrase:
                break
            await asyncio.sleep(0.01)
        assert sp is not None and sp.t_first_phrase
        assert comps.get_health_status().active_sessions == 1
        assert proc.interrupt_relay("relay-a") is True
        r1 = await asyncio.wait_for(first, 120)
        # a second utterance of the same relay now speaks normally
        r2 = await asyncio.wait_for(proc.process("relay-a", "req-2", None, 16000,
                                                 transcript_hint=HINT, pcm16=_pcm()), 120)
        await proc.close()
        return r1, r2
    r1, r2 = asyncio.run(go())
    s1 = r1.metrics["speech"]
    assert s1["interrupted"] is True
    # no further phrase was synthesised and published after the interrupt
    assert s1["phrases"] < s1["streaming"]["phrase_count"]
    assert r2.metrics["speech"]["interrupted"] is False
    assert r2.metrics["speech"]["phrases"] == r2.metrics["speech"]["streaming"]["phrase_count"]
    agg = comps.metrics.get_aggregate_metrics()
    assert agg.total_sessions == 2 and agg.interrupted_sessions == 1
    assert agg.completed_sessions == 1
    assert proc.stats["interrupted"] == 1
    assert comps.get_health_status().active_sessions == 0


def test_audio_service_interrupts_on_new_winner():
    """AudioService asks the processor to interrupt a relay's reply the moment
    that relay wins a new arbitration window."""
    from loqa_hub_amd.transport.audio_service import AudioService, UtteranceResult

    class Proc:
        def __init__(self):
            self.interrupted = []

        def interrupt_relay(self, relay_id):
            self.interrupted.append(relay_id)
            return True

        async def process(self, relay_id, request_id, audio, sr, **kw):
            return UtteranceResult(transcription="x", response_text="ok")

    async def go():
        p = Proc()
        svc = AudioService(p, window_duration=0.01, end_of_speech_wait=0.05)
        w = svc.start_arbitration_window("relay-a")
        w.relays["relay-a"].add_pcm(b"\x10\x00" * 1600)
        w.relays["relay-a"].wake_pcm += b"\x10\x00" * 1600
        w.relays["relay-a"].end_of_speech.set()
        svc.perform_arbitration(w)
        await w.relays["relay-a"].result
        return p, svc
    p, svc = asyncio.run(go())
    assert p.interrupted == ["relay-a"] and svc.stats["interrupted"] == 1
