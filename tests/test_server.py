"""Hub composition (C1/C3), skills CLI (C2), streaming + metrics APIs, and the
service-path voice processor, end to end over real sockets (HTTP + gRPC +
embedded NATS)."""
import asyncio
import io
import json
import urllib.request

import numpy as np
import pytest

from loqa_hub_amd import config as cfgmod
from loqa_hub_amd.cli import skills_cli
from loqa_hub_amd.llm.command_parser import CommandParser, OllamaBackend
from loqa_hub_amd.llm.http import create_mock_ollama
from loqa_hub_amd.llm.transcriber import TranscriptionResult
from loqa_hub_amd.server import HubServer
from loqa_hub_amd.transport.audio_proto import AudioChunk, stream_audio_stub
from loqa_hub_amd.transport.voice_processor import ServiceVoiceProcessor, float_to_pcm16


class FakeSTT:
    def __init__(self, text):
        self.text = text

    async def transcribe_with_confidence(self, audio, sr):
        return TranscriptionResult(self.text, 0.9, False, "", False)


def multi_reply(prompt):
    if "is_multi" in prompt:
        return json.dumps({"commands": [
            {"intent": "turn_on", "entities": {"device": "lights"}, "confidence": 0.9,
             "response": "Lights on"},
            {"intent": "turn_off", "entities": {"device": "fan"}, "confidence": 0.9,
             "response": "Fan off"}], "is_multi": True,
            "combined_response": "Turning on the lights and turning off the fan"})
    return json.dumps({"intent": "greeting", "entities": {}, "confidence": 0.9,
                       "response": "Hello!"})


def make_cfg(tmp_path):
    return cfgmod.load({"LOQA_DB_PATH": str(tmp_path / "hub.db"), "NATS_URL": "embedded",
                        "ARBITRATION_WINDOW_DURATION": "50ms"})


def http_get(url):
    with urllib.request.urlopen(url, timeout=10) as r:
        return r.status, r.read().decode()


def pcm(amp, n=1600):
    return (amp * np.sin(np.arange(n) / 5.0)).astype("<i2").tobytes()


async def relay(relay_id):
    yield AudioChunk(relay_id=relay_id, audio_data=pcm(8000), sample_rate=16000, is_wake_word=True)
    for i in range(3):
        await asyncio.sleep(0.01)
        yield AudioChunk(relay_id=relay_id, audio_data=pcm(8000), sample_rate=16000,
                         is_end_of_speech=i == 2)


def test_hub_server_end_to_end(tmp_path):
    grpc = pytest.importorskip("grpc")

    async def go():
        cfg = make_cfg(tmp_path)
        srv = HubServer(cfg, skills_dir=str(tmp_path / "skills"),
                        skills_config_store=str(tmp_path / "skillcfg"))
        await srv._connect_nats()
        parser = CommandParser(OllamaBackend(client=create_mock_ollama(multi_reply)))
        srv.processor = ServiceVoiceProcessor(
            FakeSTT("turn on the lights and turn off the fan"), parser, nats=srv.nats)
        await srv.start(host="127.0.0.1", http_port=0, grpc_port=0)
        try:
            base = f"http://127.0.0.1:{srv.http_port}"
            st, body = await asyncio.to_thread(http_get, base + "/health")
            assert (st, body) == (200, "ok\n")
            st, body = await asyncio.to_thread(http_get, base + "/api/skills")
            assert json.loads(body)["count"] == 1
            async with grpc.aio.insecure_channel(f"127.0.0.1:{srv.grpc_port}") as ch:
                got = [r async for r in stream_audio_stub(ch)(relay("kitchen-relay"))]
            last = got[-1]
            assert last.success and last.transcription == "turn on the lights and turn off the fan"
            # the first command's response, as audio_service.go:687-689
            assert last.response_text == "Lights on"
            st, body = await asyncio.to_thread(http_get, base + "/api/voice-events")
            ev = json.loads(body)
            assert ev["total"] == 1 and ev["events"][0]["relay_id"] == "kitchen-relay"
            assert ev["events"][0]["intent"] == "turn_on"
            st, body = await asyncio.to_thread(http_get, base + "/api/metrics")
            assert "loqa_audio_processed_total 1.0" in body and "loqa_nats_out_msgs" in body
            req = urllib.request.Request(base + "/api/streaming/health")
            with pytest.raises(urllib.error.HTTPError) as ei:
                await asyncio.to_thread(urllib.request.urlopen, req)
            assert ei.value.code == 503
            # skills CLI against the live hub
            out, err = io.StringIO(), io.StringIO()
            rc = await asyncio.to_thread(skills_cli.main, ["-hub", base, "-action", "list"], out,
                                         err)
            assert rc == 0 and "builtin.lights" in out.getvalue()
            assert "Total: 1 skills" in out.getvalue()
            out = io.StringIO()
            rc = await asyncio.to_thread(skills_cli.main, ["-hub", base, "-action", "info",
                                                           "-skill", "missing"], out, err)
            assert rc == 1 and "skill missing not found" in err.getvalue()
            rc = await asyncio.to_thread(skills_cli.main, ["-hub", base, "-action", "unload"],
                                         out, err)
            assert rc == 1 and "skill ID required for unload action" in err.getvalue()
            rc = await asyncio.to_thread(skills_cli.main, ["-hub", base, "-action", "bogus"], out,
                                         err)
            assert rc == 1 and "unknown action bogus" in err.getvalue()
        finally:
            await srv.stop()
    asyncio.run(go())


def test_streaming_api_with_components(tmp_path):
    from aiohttp import web
    from aiohttp.test_utils import TestClient, TestServer

    from loqa_hub_amd.api.streaming import StreamingHandler
    from loqa_hub_amd.streaming import StreamingComponents

    class TTS:
        async def synthesize(self, text, options=None):
            from loqa_hub_amd.llm.tts import TTSResult
            return TTSResult(b"x", "audio/wav", 1)

    async def go():
        cfg = cfgmod.load({"STREAMING_ENABLED": "false"})
        comps = await StreamingComponents.create(
            cfg, TTS(), fallback=CommandParser(OllamaBackend(client=create_mock_ollama(
                multi_reply))))
        res = await comps.process_streaming_command("hello", "s1")
        await res.collect()
        for _ in range(100):
            if comps.metrics.get_aggregate_metrics().completed_sessions:
                break
            await asyncio.sleep(0.01)
        app = web.Application()
        app.add_routes(StreamingHandler(comps).routes())
        async with TestClient(TestServer(app)) as c:
            h = await (await c.get("/api/streaming/health")).json()
            assert h["overall_health"] == "healthy" and h["parser_enabled"] is False
            m = await (await c.get("/api/streaming/metrics")).json()
            assert m["summary"]["total_sessions"] == 1
            assert isinstance(m["summary"]["average_completion"], str)
            s = await (await c.get("/api/streaming/sessions")).json()
            assert "metrics" in s and s["metrics"]["active_sessions"] == len(s["active_sessions"])
            e = await (await c.get("/api/streaming/metrics/export?include_sessions=false")).json()
            assert "recent_sessions" not in e
            assert (await c.get("/api/streaming/metrics/export?format=xml")).status == 400
        await comps.shutdown()
    asyncio.run(go())


def test_float_to_pcm16_roundtrip():
    from loqa_hub_amd.transport.audio_service import bytes_to_float32_array
    x = np.array([0, 1000, -32767, 32767], np.int16)
    back = float_to_pcm16(bytes_to_float32_array(x.tobytes()))
    assert np.array_equal(back, x)


def test_gpu_voice_processor_batches_on_cpu(tmp_path):
    """The on-device pipeline processor (tiny models on the CPU here) micro-
    batches concurrent winners into one pipeline call."""
    from loqa_hub_amd.server import build_gpu_processor

    async def go():
        cfg = cfgmod.load({"HUB_STT_MODEL": "test-whisper", "HUB_LLM_MODEL": "test-tiny",
                           "HUB_MAX_BATCH": "4", "HUB_USE_GRAPHS": "false"})
        proc = build_gpu_processor(cfg, None, device="cpu")
        rng = np.random.default_rng(0)
        audios = [rng.standard_normal(16000).astype(np.float32) * 0.1 for _ in range(3)]
        res = await asyncio.gather(*[proc.process(f"r{i}", f"q{i}", a, 16000)
                                     for i, a in enumerate(audios)])
        assert proc.stats["utterances"] == 3
        assert proc.pipeline.stats == {"stt_batches": 1, "utterances": 3}
        assert all(r.command in ("voice_command_success", "no_speech", "error",
                                 "confirmation_needed") for r in res)
    asyncio.run(go())


def test_deferred_logging_keeps_failures_and_call_time_args(monkeypatch, capsys):
    """with the async log handler, WARNING+ lines are written
    before the call returns (a process killed right after keeps them), and a
    deferred INFO line renders its args as they were at the call."""
    import logging as _logging

    from loqa_hub_amd.utils import logging as lg
    monkeypatch.setenv("LOQA_LOG_ASYNC", "1")
    root = _logging.getLogger(lg.ROOT)
    try:
        lg.initialize("info", "console")
        h = root.handlers[0]
        assert isinstance(h, lg._DeferredHandler)
        h.listener.stop()                 # nothing deferred is written from here on
        lg.get("t").error("gpu fault on %s", "rank3")
        assert "gpu fault on rank3" in capsys.readouterr().err
        box = ["before"]
        lg.get("t").info("state=%s", box)
        box[0] = "after"
        rec = h.queue.get_nowait()
        assert rec.getMessage() == "state=['before']"
        h.listener.start()                # its atexit stop() needs a running thread
    finally:
        for x in list(root.handlers):
            root.removeHandler(x)
