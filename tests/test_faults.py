"""FAULT_INJECT recovery paths on the live on-device pipeline
(tiny models on the CPU): STT failure -> error reply, LLM timeout -> parse-failed
reply without commands, NATS down -> queue failure (rollback path), TTS failure
-> text-only reply (graceful degrade)."""
import asyncio

import pytest
import torch

from loqa_hub_amd.engine.synthetic import make_batch
from loqa_hub_amd.transport.audio_service import MSG_PARSE_FAILED, MSG_STT_FAILED
from loqa_hub_amd.utils.faults import set_faults


@pytest.fixture(scope="module")
def engines():
    from loqa_hub_amd.engine.llm_engine import LLMEngine
    from loqa_hub_amd.engine.stt_engine import STTEngine
    from loqa_hub_amd.models.configs import llama_config, whisper_config
    stt = STTEngine(whisper_config("test-whisper"), torch.device("cpu"), seed=0, max_batch=4)
    llm = LLMEngine(llama_config("test-tiny"), torch.device("cpu"), seed=0, max_seqs=4,
                    max_seq_len=1024, use_graphs=False)
    return stt, llm


@pytest.fixture(autouse=True)
def _reset_faults():
    yield
    set_faults("")


def _process(engines, fault, *, nats=False, tts=None):
    from loqa_hub_amd.engine.pipeline import VoicePipeline
    from loqa_hub_amd.messaging.nats_server import NATSServer
    from loqa_hub_amd.messaging.nats_service import NATSService
    from loqa_hub_amd.transport.voice_processor import GPUVoiceProcessor

    async def main():
        srv = svc = None
        if nats:
            srv = await NATSServer().start()
            svc = NATSService(srv.url)
            await svc.connect()
        stt, llm = engines
        pipe = VoicePipeline(stt, llm, svc, min_response_tokens=2)
        proc = GPUVoiceProcessor(pipe, tts=tts, max_batch=4)
        set_faults(fault)
        utts = make_batch(0, 2, [2, 1])
        try:  # teacher-forced transcripts (random-init Whisper)
            res = await asyncio.gather(*[proc.process(u.relay_id, f"r{i}", u.pcm / 32767.0, 16000,
                                                      transcript_hint=u.text)
                                         for i, u in enumerate(utts)])
        finally:
            if svc:
                await svc.close()
            if srv:
                await srv.stop()
        return res
    return asyncio.run(main())


def test_no_fault_baseline(engines):
    res = _process(engines, "", nats=True)
    assert all(r.success and r.intents for r in res)


def test_stt_error_gives_error_reply(engines):
    res = _process(engines, "stt_error")
    assert all(r.command == "error" and r.response_text == MSG_STT_FAILED for r in res)


def test_llm_timeout_gives_parse_failed_reply(engines):
    res = _process(engines, "llm_timeout")
    assert all(not r.success and r.response_text == MSG_PARSE_FAILED for r in res)


def test_nats_down_fails_the_command_queue(engines):
    res = _process(engines, "nats_down", nats=True)
    assert all(r.intents and not r.success for r in res)


def test_tts_error_degrades_to_text(engines):
    class FakeTTS:
        async def synthesize(self, text, opts=None):
            from loqa_hub_amd.utils.faults import faults
            faults().check("tts_error")
            raise AssertionError("unreachable")
    res = _process(engines, "tts_error", nats=True, tts=FakeTTS())
    assert all(r.success and r.response_text and not r.audio for r in res)


def test_tracing_spans_recorded(engines):
    import json

    from loqa_hub_amd.utils.tracing import tracer
    tracer().clear()
    _process(engines, "", nats=True)
    summ = tracer().summary()
    for stage in ("h2d", "encode", "stt_decode", "llm", "parse", "queue"):
        assert stage in summ and summ[stage]["count"] >= 1, (stage, summ.keys())
    ev = json.loads(tracer().chrome_trace())["traceEvents"]
    assert any(e["name"] == "queue" for e in ev)
