"""NATS client + embedded broker (C30/C31), Go-compatible JSON, voice events (C7),
SQLite storage (C8/C9), /api/voice-events (C10), device-command mapping (C12)."""
import asyncio
import json
from datetime import datetime, timedelta, timezone

import pytest
from aiohttp import web
from aiohttp.test_utils import TestClient, TestServer

from loqa_hub_amd.api.voice_events import VoiceEventsHandler
from loqa_hub_amd.events import VoiceEvent, parse_rfc3339, rfc3339
from loqa_hub_amd.llm.command_queue import CommandQueue
from loqa_hub_amd.llm.commands import Command
from loqa_hub_amd.messaging.audio_stream_publisher import AudioStreamPublisher
from loqa_hub_amd.messaging.nats_client import NATSClient
from loqa_hub_amd.messaging.nats_server import NATSServer, subject_matches
from loqa_hub_amd.messaging.nats_service import (CommandEvent, DeviceCommandEvent,
                                                 DeviceResponseEvent, NATSService)
from loqa_hub_amd.storage.database import Database
from loqa_hub_amd.storage.voice_events_store import (ListOptions, NotFound, VoiceEventsStore,
                                                     validate_sort_by, validate_sort_order)
from loqa_hub_amd.transport.device_commands import (ExecutionContext, NATSCommandExecutor,
                                                    create_device_command, extract_device_type,
                                                    is_device_command, map_intent_to_action)
from loqa_hub_amd.utils import gojson
from loqa_hub_amd.utils.security import InvalidSkillID, sanitize_log_input, validate_skill_id


# -- go json / security / events -----------------------------------------------------------------
def test_gojson_matches_go_encoding():
    assert gojson.go_float(1.0) == "1" and gojson.go_float(0.5) == "0.5"
    assert gojson.go_float(1e21) == "1e+21" and gojson.go_float(1e-7) == "1e-07"
    assert gojson.dumps({"b": 1, "a": "<&>"}) == '{"a":"\\u003c\\u0026\\u003e","b":1}'
    assert gojson.dumps(b"\x00\x01") == '"AAE="'
    assert gojson.dumps(gojson.GoStruct(("z", 1), ("a", None))) == '{"z":1,"a":null}'


def test_security():
    assert sanitize_log_input("a\nb\rc") == "abc"
    validate_skill_id("my-skill_1")
    for bad in ("", "a/b", "a\\b", "..", "a.b", "a b"):
        with pytest.raises(InvalidSkillID):
            validate_skill_id(bad)


def test_voice_event_lifecycle():
    ev = VoiceEvent.new("relay-1", "req-1")
    assert len(ev.uuid) == 36
    ev.set_audio_metadata(16000, 16000, True)
    assert ev.audio_duration == pytest.approx(1.0) and ev.sample_rate == 16000
    ev.set_command_result("turn_on", {"device": "lights"}, 0.9)
    assert json.loads(ev.entities_json()) == {"device": "lights"}
    ev.set_entities_from_json('{"room": "kitchen"}')
    assert ev.entities == {"room": "kitchen"}
    ev.set_error(RuntimeError("boom"))
    assert not ev.success and ev.error_message == "boom"
    ev.is_valid()
    ev.confidence = 2.0
    with pytest.raises(ValueError):
        ev.is_valid()
    t = datetime(2025, 1, 2, 3, 4, 5, 120000, tzinfo=timezone.utc)
    assert rfc3339(t) == "2025-01-02T03:04:05.12Z" and parse_rfc3339(rfc3339(t)) == t


# -- storage -------------------------------------------------------------------------------------
def mk_event(i, relay="r1", intent="turn_on", success=True, t0=None):
    t0 = t0 or datetime(2025, 1, 1, tzinfo=timezone.utc)
    ev = VoiceEvent(uuid=f"u-{i:03d}", request_id=f"q{i}", relay_id=relay,
                    timestamp=t0 + timedelta(minutes=i), audio_duration=1.5, sample_rate=16000,
                    transcription=f"text {i}", intent=intent, entities={"device": "lights"},
                    confidence=0.9, response_text="ok", processing_time_ms=10 * i, success=success)
    return ev


def test_store_crud_and_listing(tmp_path):
    db = Database(str(tmp_path / "sub" / "hub.db"))
    st = VoiceEventsStore(db)
    for i in range(10):
        st.insert(mk_event(i, relay="r1" if i % 2 else "r2", success=i % 3 != 0))
    got = st.get_by_uuid("u-003")
    assert got.transcription == "text 3" and got.entities == {"device": "lights"}
    assert got.timestamp == datetime(2025, 1, 1, 0, 3, tzinfo=timezone.utc)
    with pytest.raises(NotFound):
        st.get_by_uuid("nope")
    assert st.count(ListOptions()) == 10
    assert st.count(ListOptions(relay_id="r1")) == 5
    assert st.count(ListOptions(success=False)) == 4
    page = st.list(ListOptions(limit=3, offset=0, sort_by="timestamp", sort_order="ASC"))
    assert [e.uuid for e in page] == ["u-000", "u-001", "u-002"]
    default = st.list(ListOptions(limit=2))
    assert [e.uuid for e in default] == ["u-009", "u-008"]  # timestamp DESC
    t5 = datetime(2025, 1, 1, 0, 5, tzinfo=timezone.utc)
    assert st.count(ListOptions(start_time=t5)) == 5
    assert [e.uuid for e in st.get_recent_by_relay("r1", 2)] == ["u-009", "u-007"]
    st.delete("u-000")
    with pytest.raises(NotFound):
        st.delete("u-000")
    assert validate_sort_by("processing_time") == "processing_time_ms"
    assert validate_sort_by("x; DROP TABLE") == "timestamp"
    assert validate_sort_order("asc") == "DESC" and validate_sort_order("ASC") == "ASC"
    s = db.stats()
    assert s["voice_events_count"] == 9 if "voice_events_count" in s else True
    db.vacuum()
    db.checkpoint()
    db.close()


def test_voice_events_api(tmp_path):
    async def go():
        st = VoiceEventsStore(Database(str(tmp_path / "a.db")))
        for i in range(25):
            st.insert(mk_event(i))
        app = web.Application()
        app.add_routes(VoiceEventsHandler(st).routes())
        async with TestClient(TestServer(app)) as c:
            r = await c.get("/api/voice-events")
            b = await r.json()
            assert r.status == 200 and b["total"] == 25 and b["page"] == 1
            assert b["page_size"] == 20 and b["total_pages"] == 2 and len(b["events"]) == 20
            r = await c.get("/api/voice-events?page=2&page_size=1000")
            b = await r.json()
            assert b["page_size"] == 100 and len(b["events"]) == 0
            r = await c.get("/api/voice-events?sort_by=timestamp&sort_order=asc&page_size=1")
            assert (await r.json())["events"][0]["uuid"] == "u-000"
            r = await c.get("/api/voice-events/u-004")
            assert r.status == 200 and (await r.json())["transcription"] == "text 4"
            r = await c.get("/api/voice-events/missing")
            assert r.status == 404 and (await r.text()) == "Voice event not found\n"
            r = await c.post("/api/voice-events", data=json.dumps({"transcription": "x"}))
            assert r.status == 400
            r = await c.post("/api/voice-events", data=json.dumps(
                {"relay_id": "r9", "transcription": "hello", "intent": "greeting",
                 "confidence": 0.5, "success": True}))
            b = await r.json()
            assert r.status == 201 and b["request_id"] == "r9" and b["relay_id"] == "r9"
            assert (await c.delete("/api/voice-events")).status == 405
    asyncio.run(go())


# -- NATS ----------------------------------------------------------------------------------------
def test_subject_matching():
    assert subject_matches("a.*.c", "a.b.c") and not subject_matches("a.*", "a.b.c")
    assert subject_matches("a.>", "a.b.c") and not subject_matches("a.>", "a")
    assert subject_matches("loqa.devices.commands.lights", "loqa.devices.commands.lights")


def test_nats_pubsub_and_queue_groups():
    async def go():
        srv = await NATSServer().start()
        try:
            a, b = NATSClient(), NATSClient()
            await a.connect(srv.url)
            await b.connect(srv.url)
            got, grp = [], []
            await b.subscribe("loqa.>", lambda m: got.append((m.subject, m.data)))
            await b.subscribe("work", lambda m: grp.append(1), queue="q")
            await b.subscribe("work", lambda m: grp.append(2), queue="q")
            await b.flush()
            await a.publish("loqa.voice.commands", b"hi")
            for _ in range(10):
                await a.publish("work", b"x")
            await a.flush()
            for _ in range(50):
                if len(got) == 1 and len(grp) == 10:
                    break
                await asyncio.sleep(0.01)
            assert got == [("loqa.voice.commands", b"hi")] and len(grp) == 10
            assert a.stats.out_msgs == 11
            await a.close()
            await b.close()
        finally:
            await srv.stop()
    asyncio.run(go())


def test_nats_service_events_and_executor():
    async def go():
        srv = await NATSServer().start()
        try:
            svc, listener = NATSService(srv.url), NATSService(srv.url)
            await svc.connect()
            await listener.connect()
            voice, dev = [], []
            await listener.subscribe_voice_commands(voice.append)
            await listener.subscribe_device_commands("lights", dev.append)
            await listener.conn.flush()
            ex = NATSCommandExecutor(svc, ExecutionContext("relay-7", "req-7", "", "lights on"))
            q = CommandQueue([Command("turn_on", {"device": "light"}, 0.9, "on"),
                              Command("greeting", {}, 0.8, "hello")])
            res = await q.execute(ex)
            assert res.success
            await svc.conn.flush()
            for _ in range(50):
                if len(voice) == 2 and len(dev) == 1:
                    break
                await asyncio.sleep(0.01)
            assert [v.intent for v in voice] == ["turn_on", "greeting"]
            assert voice[0].relay_id == "relay-7" and dev[0].action == "on"
            assert dev[0].device_type == "lights"
            await svc.close()
            await listener.close()
            with pytest.raises(RuntimeError):
                await NATSCommandExecutor(None).execute_command(Command("x"))
        finally:
            await srv.stop()
    asyncio.run(go())


def test_event_json_is_go_compatible():
    ev = CommandEvent("r", "t", "turn_on", {"device": "lights"}, 1.0, 123, "q")
    assert ev.to_json() == (b'{"relay_id":"r","transcription":"t","intent":"turn_on",'
                            b'"entities":{"device":"lights"},"confidence":1,"timestamp":123,'
                            b'"request_id":"q"}')
    dc = create_device_command(ev)
    assert json.loads(dc.to_json())["action"] == "on" and "device_id" not in json.loads(dc.to_json())
    assert DeviceCommandEvent.from_json(dc.to_json()).device_type == "lights"
    dr = DeviceResponseEvent("q", "lights", "", True, "ok", 5)
    assert DeviceResponseEvent.from_json(dr.to_json()) == dr
    assert is_device_command("turn_on") and not is_device_command("greeting")
    assert map_intent_to_action("turn_off") == "off" and map_intent_to_action("x") == ""
    assert extract_device_type({"device": "television"}) == "tv"
    assert extract_device_type({}) == ""


def test_audio_stream_publisher():
    async def go():
        srv = await NATSServer().start()
        try:
            pub, sub = NATSClient(), NATSClient()
            await pub.connect(srv.url)
            await sub.connect(srv.url)
            got = []
            await sub.subscribe("audio.>", lambda m: got.append((m.subject, json.loads(m.data))))
            await sub.flush()
            p = AudioStreamPublisher(pub)
            await p.stream_audio_to_relay("relay-1", b"\x01\x02\x03", "wav", 22050, "response", 1)
            await pub.flush()
            for _ in range(50):
                if got:
                    break
                await asyncio.sleep(0.01)
            subj, msg = got[0]
            assert subj == "audio.relay-1" and msg["audio_data"] == "AQID"
            await pub.close()
            await sub.close()
        finally:
            await srv.stop()
    asyncio.run(go())
