"""Streaming subsystem (C20-C24) and the STT/TTS HTTP clients (C14-C16); cases
follow the reference's ``streaming_test.go`` / ``openai_tts_client_test.go`` /
``stt_client_test.go``."""
import asyncio
import json
import struct

import numpy as np
import pytest

from loqa_hub_amd import config as cfgmod
from loqa_hub_amd.llm.command_parser import CommandParser, OllamaBackend
from loqa_hub_amd.llm.http import HTTPResponse, MockHTTPClient, create_mock_ollama
from loqa_hub_amd.llm.stt_client import STTClient, float32_to_wav
from loqa_hub_amd.llm.tts import OpenAITTSClient, TTSOptions, TTSResult
from loqa_hub_amd.streaming import (Chan, OllamaStreamingBackend, PhraseBuffer,
                                    StreamingAudioPipeline, StreamingCommandParser,
                                    StreamingComponents, StreamingInterruptHandler,
                                    StreamingMetricsCollector)
from loqa_hub_amd.streaming.parser import StreamingMetrics

CMD = {"intent": "turn_on", "entities": {"device": "lights", "location": "kitchen"},
       "confidence": 0.95, "response": "Turning on the kitchen lights. Done!"}


def ndjson_tokens(text, n=7):
    pieces = [text[i:i + n] for i in range(0, len(text), n)]
    lines = [json.dumps({"response": p, "done": False}) for p in pieces]
    lines.append(json.dumps({"response": "", "done": True}))
    return ("\n".join(lines) + "\n").encode()


def mock_stream_client(text):
    return MockHTTPClient({"/api/generate": HTTPResponse(200, ndjson_tokens(text))})


class FakeTTS:
    def __init__(self, delays=None, fail=()):
        self.delays, self.fail, self.calls = delays or {}, set(fail), []

    async def synthesize(self, text, options=None):
        self.calls.append(text)
        await asyncio.sleep(self.delays.get(text, 0.0))
        if text in self.fail:
            raise RuntimeError("tts down")
        return TTSResult(text.encode(), "audio/wav", len(text))

    async def get_available_voices(self):
        return ["af_bella"]

    async def close(self):
        pass


def test_phrase_buffer_boundaries():
    pb = PhraseBuffer()
    assert pb.add_token("Turning on") == ""
    assert pb.add_token(" the lights.") == "Turning on the lights."
    assert pb.add_token("Yes") == "" and pb.add_token(", and") == "Yes, and"
    assert pb.add_token(" more") == "" and pb.flush() == "more" and pb.flush() == ""
    pb = PhraseBuffer(max_tokens=3)
    assert [pb.add_token(t) for t in ("a", "b", "c")] == ["", "", "abc"]


def test_streaming_parser_ollama_ndjson():
    async def go():
        text = json.dumps(CMD)
        p = StreamingCommandParser(OllamaStreamingBackend("http://x", "m", mock_stream_client(text)),
                                   None, True)
        res = await p.parse_command_streaming("turn on the kitchen lights")
        toks, phrases, cmd, err = await res.collect()
        assert err is None and "".join(toks) == text
        assert cmd.intent == "turn_on" and cmd.entities["location"] == "kitchen"
        assert "".join(phrases).replace(" ", "") == text.replace(" ", "")
        assert res.metrics.token_count == len(toks) and res.metrics.completion_time > 0
    asyncio.run(go())


def test_streaming_parser_disabled_and_empty():
    async def go():
        fb = CommandParser(OllamaBackend(client=create_mock_ollama(json.dumps(CMD))))
        p = StreamingCommandParser(None, fb, enabled=False)
        toks, phrases, cmd, _ = await (await p.parse_command_streaming("lights on")).collect()
        assert toks == [CMD["response"]] and cmd.intent == "turn_on"
        p2 = StreamingCommandParser(OllamaStreamingBackend("http://x", "m", mock_stream_client("")),
                                    fb, True)
        _, _, cmd, _ = await (await p2.parse_command_streaming("")).collect()
        assert cmd.response == "I didn't hear anything."
        with pytest.raises(RuntimeError):
            await p.test_streaming_connection()
    asyncio.run(go())


def test_streaming_parser_bad_json_reports_error():
    async def go():
        p = StreamingCommandParser(OllamaStreamingBackend("http://x", "m",
                                                          mock_stream_client("not json at all")),
                                   None, True)
        _, _, cmd, err = await (await p.parse_command_streaming("x")).collect()
        assert cmd is None and "parsing final command" in str(err)
    asyncio.run(go())


def test_audio_pipeline_reorders_and_marks_last():
    async def go():
        tts = FakeTTS(delays={"one": 0.05, "two": 0.0, "three": 0.02}, fail={"bad"})
        pipe = StreamingAudioPipeline(tts, max_concurrent=3)
        phrases = Chan(10)
        pc = pipe.start_pipeline("s1", phrases)
        with pytest.raises(ValueError):
            pipe.start_pipeline("s1", Chan(1))
        for p in ("one", "two", "bad", "", "three"):
            await phrases.put(p)
        phrases.close()
        chunks = []
        async for c in pc.audio_chunks:
            chunks.append(c)
            if c.is_last:
                break
        assert [c.phrase for c in chunks] == ["one", "two", "three", ""]
        assert chunks[-1].is_last and chunks[-1].sequence_id == 4
        m = pipe.get_pipeline_metrics("s1")
        assert m.total_phrases == 4 and m.synthesized_phrases == 3 and m.failed_synthesis == 1
        await pipe.stop_pipeline("s1")
        assert pipe.get_active_pipelines() == []
    asyncio.run(go())


def test_interrupt_handler():
    async def go():
        h = StreamingInterruptHandler(0.05, 0.1)
        cancelled = []
        h.register_session("a", cancel=lambda: cancelled.append("a"))
        h.register_session("b")
        assert sorted(h.get_active_session_ids()) == ["a", "b"]
        t = h.interrupt_session("a", "user_request")
        assert h.interrupt_session("a", "user_request") is None  # idempotent
        assert h.get_session_metrics().interrupt_reasons == {"user_request": 1}
        await t
        assert h.get_active_session_ids() == ["b"]
        await h.shutdown()
        assert h.get_active_session_ids() == []
        assert h.interrupt_session("zzz", "x") is None
    asyncio.run(go())


def test_metrics_collector():
    mc = StreamingMetricsCollector(True)
    assert mc.assess_health_status() == "unknown"
    mc.record_session_start("s")
    m = StreamingMetrics(start_time=100.0, first_token_time=100.2, first_phrase_time=100.4,
                         completion_time=101.0, token_count=50, phrase_count=3)
    mc.record_session_metrics("s", m)
    a = mc.get_aggregate_metrics()
    assert a.completed_sessions == 1 and a.average_first_token == pytest.approx(0.2)
    assert a.throughput_tokens_per_sec == pytest.approx(50.0)
    assert mc.assess_health_status() == "healthy"
    mc.record_session_start("t")
    mc.record_session_metrics("t", StreamingMetrics(start_time=1.0, interrupt_count=1))
    assert mc.get_aggregate_metrics().error_rate == pytest.approx(0.5)
    assert mc.assess_health_status() == "critical"
    rep = json.loads(mc.export_metrics())
    assert rep["health_status"] == "critical" and rep["summary"]["total_sessions"] == 2
    assert rep["summary"]["average_first_token"] == 200_000_000
    off = StreamingMetricsCollector(False)
    assert off.generate_performance_report()["health_status"] == "disabled"


def test_components_end_to_end():
    async def go():
        cfg = cfgmod.load({"STREAMING_ENABLED": "true", "STREAMING_INTERRUPT_TIMEOUT": "100ms"})
        client = mock_stream_client(json.dumps(CMD))
        comps = await StreamingComponents.create(cfg, FakeTTS(), http_client=client)
        assert comps.interrupt_handler.force_timeout == pytest.approx(0.2)
        res = await comps.process_streaming_command("turn on the kitchen lights", "sess-1")
        _, phrases, cmd, err = await res.collect()
        assert err is None and cmd.intent == "turn_on"
        for _ in range(100):
            if comps.metrics.get_aggregate_metrics().completed_sessions:
                break
            await asyncio.sleep(0.01)
        assert comps.metrics.get_aggregate_metrics().completed_sessions == 1
        h = comps.get_health_status()
        assert h.parser_enabled and h.overall_health == "healthy"
        cfg2 = cfgmod.load({"STREAMING_ENABLED": "false", "STREAMING_AUDIO_CONCURRENCY": "5"})
        comps.update_configuration(cfg2)
        assert not comps.parser.enabled and comps.audio_pipeline.max_concurrent == 5
        await comps.shutdown()
    asyncio.run(go())


def test_stt_client_request_format():
    async def go():
        client = MockHTTPClient({"/health": HTTPResponse(200, b"ok"),
                                 "/v1/audio/transcriptions": HTTPResponse(
                                     200, b'{"text": "Hey Loqa turn on the lights"}')})
        stt = await STTClient.create("http://stt:8000", "es", client=client)
        audio = np.linspace(-1, 1, 1600).astype(np.float32)
        r = await stt.transcribe_with_confidence(audio, 16000)
        assert r.text == "turn on the lights" and r.wake_word_detected
        method, url, body = client.requests[-1]
        assert url == "http://stt:8000/v1/audio/transcriptions"
        for field, val in (("model", "tiny"), ("language", "es"), ("temperature", "0.0"),
                           ("response_format", "json")):
            assert f'name="{field}"\r\n\r\n{val}\r\n'.encode() in body
        assert b'filename="audio.wav"' in body
        with pytest.raises(ValueError):
            await stt.transcribe(np.zeros(0, np.float32), 16000)
        bad = MockHTTPClient({"/health": HTTPResponse(503)})
        with pytest.raises(ConnectionError):
            await STTClient.create("http://stt:8000", client=bad)
    asyncio.run(go())


def test_float32_wav_header():
    w = float32_to_wav(np.array([0.5, -0.25], np.float32), 16000)
    assert w[:4] == b"RIFF" and w[8:12] == b"WAVE"
    fmt = struct.unpack("<IHHIIHH", w[16:36])
    assert fmt == (16, 3, 1, 16000, 64000, 4, 32)
    assert struct.unpack("<I", w[40:44])[0] == 8 and np.frombuffer(w[44:], "<f4").tolist() == [0.5, -0.25]


def test_tts_client():
    async def go():
        cfg = cfgmod.load({"TTS_MAX_CONCURRENT": "1", "TTS_NORMALIZE": "false"}).tts
        client = MockHTTPClient({"/audio/voices": HTTPResponse(200, b'{"voices": ["af_bella"]}'),
                                 "/audio/speech": HTTPResponse(200, b"RIFFdata",
                                                               {"Content-Type": "audio/wav"})})
        tts = await OpenAITTSClient.create(cfg, client=client)
        r = await tts.synthesize("hello")
        assert r.audio == b"RIFFdata" and r.content_type == "audio/wav"
        body = json.loads(client.requests[-1][2])
        assert body == {"model": "tts-1", "input": "hello", "voice": "af_bella",
                        "response_format": "wav", "speed": 1.0,
                        "normalization_options": {"normalize": False}}
        body2 = tts.build_request("x", TTSOptions("v2", 1.5, "mp3", True))
        assert "normalization_options" not in body2 and body2["voice"] == "v2"
        assert await tts.get_available_voices() == ["af_bella"]
        n = len(client.requests)
        await tts.get_available_voices()
        assert len(client.requests) == n  # cached
        with pytest.raises(ValueError):
            await tts.synthesize("")
        with pytest.raises(ValueError):
            OpenAITTSClient(cfgmod.load({"TTS_URL": ""}).tts if False else
                            type("C", (), {"url": ""})())
    asyncio.run(go())


def test_gpu_streaming_backend_tokens_cpu():
    """GPUStreamingBackend over the local constrained decode (CPU engine):
    tokens stream per decode step and the parser's final command parses."""
    import torch

    from loqa_hub_amd.engine.llm_engine import LLMEngine
    from loqa_hub_amd.models.configs import llama_config
    from loqa_hub_amd.streaming.parser import GPUStreamingBackend, StreamingCommandParser
    eng = LLMEngine(llama_config("test-tiny"), torch.device("cpu"), max_seqs=4, max_seq_len=512)

    async def go():
        p = StreamingCommandParser(GPUStreamingBackend(eng), None, max_tokens_per_phrase=4)
        res = await p.parse_command_streaming("turn on the kitchen lights")
        toks = [t async for t in res.token_stream]
        cmd = await asyncio.wait_for(res.final_command.get(), 30)
        return toks, cmd, res.metrics
    toks, cmd, m = asyncio.run(go())
    assert len(toks) > 3 and m.token_count == len(toks) and m.phrase_count >= 1
    assert cmd.intent
