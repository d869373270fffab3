"""The served hub on the on-device pipeline, end to end (SURVEY §3.2 hot path,
VERDICT r2 #2-#4), on the CPU engines (the same code runs on the MI355X in
``tests/test_engine_gpu.py::test_hub_server_gpu_served``):

relay gRPC stream -> arbitration -> Whisper STT -> ONE constrained decode ->
command queue (NATS ``loqa.voice.commands``) -> streaming-predictive bridge on
that decode -> progressive VITS speech of the reply field, phrase by phrase on
NATS ``audio.<relay>`` -> voice event in SQLite.
"""
import asyncio
import base64
import json
import urllib.request

import numpy as np
import pytest

from loqa_hub_amd import config as cfgmod
from loqa_hub_amd.engine.grammar import INTENTS
from loqa_hub_amd.server import HubServer, build_gpu_processor

HINT = "hey loqa turn on the kitchen lights and then play some jazz"


def _pcm(n=16000):
    t = np.arange(n) / 16000.0
    return (6000 * np.sin(2 * np.pi * 220 * t)).astype("<i2").tobytes()


async def _relay(relay_id):
    from loqa_hub_amd.transport.audio_proto import AudioChunk
    yield AudioChunk(relay_id=relay_id, audio_data=_pcm(), sample_rate=16000, is_wake_word=True)
    for i in range(2):
        await asyncio.sleep(0.01)
        yield AudioChunk(relay_id=relay_id, audio_data=_pcm(), sample_rate=16000,
                         is_end_of_speech=i == 1)


def _get(url):
    with urllib.request.urlopen(url, timeout=20) as r:
        return r.status, r.read().decode()


def _served(tmp_path, device, *, streaming: bool, llm="test-tiny", stt="test-whisper",
            tts_model="test-vits", dp: int = 0, relays=("kitchen-relay",)):
    """Serve ``relays`` (one utterance each, concurrently) through a hub on the
    GPU voice processor (``dp`` = 0) or a data-parallel front end over ``dp``
    spawned workers that each build the real per-GPU composition."""
    grpc = pytest.importorskip("grpc")
    from loqa_hub_amd.messaging.nats_client import NATSClient
    from loqa_hub_amd.transport.audio_proto import stream_audio_stub

    async def go():
        env = {"LOQA_DB_PATH": str(tmp_path / "hub.db"), "NATS_URL": "embedded",
               "ARBITRATION_WINDOW_DURATION": "50ms", "HUB_STT_MODEL": stt,
               "HUB_LLM_MODEL": llm, "HUB_MAX_BATCH": "4", "HUB_TTS_MODEL": tts_model,
               "STREAMING_ENABLED": "true" if streaming else "false"}
        if len(relays) > 1:
            env["ARBITRATION_SCOPE"] = "per_relay_group"
        cfg = cfgmod.load(env)
        srv = HubServer(cfg, skills_dir=str(tmp_path / "skills"),
                        skills_config_store=str(tmp_path / "skillcfg"),
                        transcript_hints=lambda relay: HINT)
        await srv._connect_nats()
        if dp:
            from loqa_hub_amd.server import build_dp_processor
            srv.processor = await build_dp_processor(
                cfg, dp, srv.nats.url, device=device, skills_dir=str(tmp_path / "skills"),
                skills_config_store=str(tmp_path / "skillcfg"), heartbeat_s=0.2)
        else:
            from loqa_hub_amd.engine.tts_engine import VitsTTSEngine
            from loqa_hub_amd.models.configs import vits_config
            tts = VitsTTSEngine(vits_config(tts_model), device)
            srv.processor = await asyncio.to_thread(build_gpu_processor, cfg, srv.nats, device,
                                                    tts, skills=srv.skills)
        await srv.start(host="127.0.0.1", http_port=0, grpc_port=0)
        audio_msgs, cmd_msgs = {r: [] for r in relays}, []
        sub = NATSClient(name="test-relay")
        await sub.connect(srv.nats.url)
        for r in relays:
            await sub.subscribe(f"audio.{r}", lambda m, r=r: audio_msgs[r].append(json.loads(m.data)))
        await sub.subscribe("loqa.voice.commands", lambda m: cmd_msgs.append(json.loads(m.data)))
        await sub.flush()
        try:
            async with grpc.aio.insecure_channel(f"127.0.0.1:{srv.grpc_port}") as ch:
                async def one(r):
                    return [x async for x in stream_audio_stub(ch)(_relay(r))]
                got = await asyncio.gather(*[one(r) for r in relays])
            await asyncio.sleep(0.3)
            await sub.flush()
            base = f"http://127.0.0.1:{srv.http_port}"
            st, body = await asyncio.to_thread(_get, base + "/api/voice-events")
            events = json.loads(body)["events"]
            st, metrics = await asyncio.to_thread(_get, base + "/api/metrics")
            routes = {}
            for route in ("health", "metrics", "sessions", "metrics/export"):
                routes[route] = await asyncio.to_thread(_get_status, base + "/api/streaming/" + route)
            stats = dict(srv.processor.stats)
            if dp:
                stats["dp_workers"] = [w["rank"] for w in srv.processor.metrics()["workers"]
                                       if w["done"] > 0]
            return dict(zip(relays, got)), audio_msgs, cmd_msgs, events, stats, metrics, routes
        finally:
            await sub.close()
            await srv.stop()
    return asyncio.run(go())


def _get_status(url):
    try:
        with urllib.request.urlopen(url, timeout=20) as r:
            return r.status, json.loads(r.read().decode())
    except urllib.error.HTTPError as e:
        return e.code, None


def _check_served(got, audio, cmds, events, stats, metrics, routes, *, streaming, relays):
    for r in relays:
        last = got[r][-1]
        assert last.command == "voice_command_success" and last.success, (r, last)
        assert last.transcription == "turn on the kitchen lights and then play some jazz"
        assert last.response_audio[:4] == b"RIFF" and last.audio_duration > 0
        # reply audio on NATS audio.<relay>: WAV phrases (progressive) or one file
        assert audio[r] and all(base64.b64decode(m["audio_data"])[:4] == b"RIFF" for m in audio[r])
        assert all(m["sample_rate"] == 22050 and m["message_type"] == "response" for m in audio[r])
        if not streaming:
            assert len(audio[r]) == 1
    # both commands of every utterance went out on the bus (compound splitter)
    assert len(cmds) == 2 * len(relays)
    assert sorted(c["relay_id"] for c in cmds) == sorted(r for r in relays for _ in range(2))
    assert all(c["transcription"] == got[c["relay_id"]][-1].transcription for c in cmds)
    n = len(relays)
    if streaming:
        assert stats["progressive"] == n and stats["first_audio_n"] == n
        # the first phrase went to synthesis while the decode was still running
        # (the GPU variant also asserts its audio was published by then)
        assert stats["phrase_before_decode_done"] == n
    # the voice events record the decodes' parses
    assert len(events) == n
    for ev in events:
        assert ev["intent"] in INTENTS and ev["success"]
        assert ev["intent"] in [c["intent"] for c in cmds if c["relay_id"] == ev["relay_id"]]
    # the bridge ran on the shared decode (no fallback)
    assert stats["bridge_sessions"] == n and stats["bridge_fallback"] == 0
    assert f"loqa_audio_processed_total {float(n)}" in metrics
    # the streaming subsystem is composed into the hub (streaming_constructor.go:38-126)
    if streaming:
        assert all(st == 200 for st, _ in routes.values()), routes
        summary = routes["metrics"][1]["summary"]
        assert summary["total_sessions"] == n and summary["completed_sessions"] == n
        assert routes["health"][1]["overall_health"] == "healthy"
    else:
        assert all(st == 503 for st, _ in routes.values()), routes


@pytest.mark.parametrize("streaming", [True, False])
def test_hub_served_cpu(tmp_path, streaming):
    res = _served(tmp_path, "cpu", streaming=streaming)
    _check_served(*res, streaming=streaming, relays=("kitchen-relay",))


@pytest.mark.parametrize("streaming", [True, False])
def test_hub_served_dp_cpu(tmp_path, streaming):
    """The served DP hub (BASELINE config 4's serving path) does what the
    1-GPU hub does: two spawned workers, each building the real per-GPU
    composition (``dp_serving._build_worker_processor``) on the CPU engines."""
    relays = ("kitchen-relay", "bedroom-relay")
    res = _served(tmp_path, "cpu", streaming=streaming, dp=2, relays=relays)
    _check_served(*res, streaming=streaming, relays=relays)
    assert sorted(res[4]["dp_workers"]) == [0, 1]      # both workers served one


def test_hub_served_dp8_cpu(tmp_path):
    """The served DP hub at the driver's 8-rank width: eight
    spawned workers, each the real per-GPU composition on the CPU engines
    (tiny models), eight relays in their own groups - every worker is up,
    every relay is answered and every utterance is a voice event."""
    relays = tuple(f"relay-{i}" for i in range(8))
    res = _served(tmp_path, "cpu", streaming=False, dp=8, relays=relays)
    _check_served(*res, streaming=False, relays=relays)
    assert len(res[4]["dp_workers"]) == 8
