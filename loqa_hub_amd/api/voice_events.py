"""``/api/voice-events`` HTTP surface (``internal/api/voice_events.go``).

GET  /api/voice-events        page (1), page_size (20, clamped [1,100]), relay_id,
                              intent, success, start_time/end_time (RFC3339),
                              sort_by, sort_order (upper-cased)
                              -> {events,total,page,page_size,total_pages}
POST /api/voice-events        201 + event; relay_id required; request_id
                              defaults to relay_id
GET  /api/voice-events/{id}   404 "Voice event not found" when missing
Bodies are encoded byte-compatibly with Go's json.Encoder (field order of the
Go structs, trailing newline); errors are Go ``http.Error`` text bodies.
"""
from __future__ import annotations

import asyncio
import json
import logging

from aiohttp import web

from ..events import VoiceEvent, parse_rfc3339, rfc3339
from ..storage.voice_events_store import ListOptions, NotFound, VoiceEventsStore
from ..utils import gojson

log = logging.getLogger("loqa.api")

_TRUE = {"1", "t", "T", "true", "TRUE", "True"}
_FALSE = {"0", "f", "F", "false", "FALSE", "False"}


def http_error(msg: str, status: int) -> web.Response:
    """Go's http.Error: text/plain body with a trailing newline."""
    return web.Response(status=status, text=msg + "\n", content_type="text/plain",
                        charset="utf-8", headers={"X-Content-Type-Options": "nosniff"})


def go_json_response(obj, status: int = 200) -> web.Response:
    return web.Response(status=status, text=gojson.dumps(obj) + "\n", content_type="application/json")


def event_struct(ev: VoiceEvent) -> gojson.GoStruct:
    f = [("uuid", ev.uuid), ("request_id", ev.request_id), ("relay_id", ev.relay_id),
         ("timestamp", rfc3339(ev.timestamp)), ("audio_duration", float(ev.audio_duration)),
         ("sample_rate", int(ev.sample_rate)), ("wake_word_detected", bool(ev.wake_word_detected)),
         ("transcription", ev.transcription), ("intent", ev.intent), ("entities", ev.entities),
         ("confidence", float(ev.confidence)), ("response_text", ev.response_text),
         ("processing_time_ms", int(ev.processing_time_ms)), ("success", bool(ev.success))]
    if ev.error_message:
        f.append(("error_message", ev.error_message))
    return gojson.GoStruct(*f)


def parse_int_param(v: str | None, default: int) -> int:
    if not v:
        return default
    try:
        return int(v, 10) if v.lstrip("+-").isdigit() else default
    except ValueError:
        return default


class VoiceEventsHandler:
    def __init__(self, store: VoiceEventsStore):
        self.store = store

    def routes(self) -> list[web.RouteDef]:
        return [web.route("*", "/api/voice-events", self.handle_voice_events),
                web.route("*", "/api/voice-events/{tail:.*}", self.handle_voice_event_by_id)]

    async def handle_voice_events(self, req: web.Request) -> web.StreamResponse:
        if req.method == "GET":
            return await self.list_voice_events(req)
        if req.method == "POST":
            return await self.create_voice_event(req)
        return http_error("Method not allowed", 405)

    async def handle_voice_event_by_id(self, req: web.Request) -> web.StreamResponse:
        if req.method != "GET":
            return http_error("Method not allowed", 405)
        parts = req.match_info.get("tail", "").split("/")
        if not parts or parts[0] == "":
            return http_error("Event ID is required", 400)
        return await self.get_voice_event(parts[0])

    async def list_voice_events(self, req: web.Request) -> web.Response:
        q = req.rel_url.query
        page = parse_int_param(q.get("page"), 1)
        page_size = parse_int_param(q.get("page_size"), 20)
        page_size = min(page_size, 100)
        page_size = max(page_size, 1)
        page = max(page, 1)
        opts = ListOptions(relay_id=q.get("relay_id", ""), intent=q.get("intent", ""),
                           limit=page_size, offset=(page - 1) * page_size,
                           sort_by=q.get("sort_by", ""), sort_order=q.get("sort_order", "").upper())
        s = q.get("success", "")
        if s in _TRUE:
            opts.success = True
        elif s in _FALSE:
            opts.success = False
        for key, attr in (("start_time", "start_time"), ("end_time", "end_time")):
            v = q.get(key, "")
            if v:
                try:
                    setattr(opts, attr, parse_rfc3339(v))
                except ValueError:
                    pass
        try:
            total = await asyncio.to_thread(self.store.count, opts)
            events = await asyncio.to_thread(self.store.list, opts)
        except Exception as e:
            log.error("failed to list voice events: %s", e)
            return http_error("Internal server error", 500)
        total_pages = (total + page_size - 1) // page_size
        body = gojson.GoStruct(("events", [event_struct(e) for e in events]), ("total", total),
                               ("page", page), ("page_size", page_size), ("total_pages", total_pages))
        return go_json_response(body)

    async def create_voice_event(self, req: web.Request) -> web.Response:
        try:
            d = json.loads(await req.read())
            if not isinstance(d, dict):
                raise ValueError
        except ValueError:
            return http_error("Invalid JSON", 400)
        relay = d.get("relay_id") or ""
        if not isinstance(relay, str) or relay == "":
            return http_error("relay_id is required", 400)
        request_id = d.get("request_id") or relay
        ev = VoiceEvent.new(relay, str(request_id))
        ev.set_transcription(str(d.get("transcription") or ""))
        ents = d.get("entities") or {}
        ev.set_command_result(str(d.get("intent") or ""), {str(k): str(v) for k, v in ents.items()}
                              if isinstance(ents, dict) else {}, float(d.get("confidence") or 0.0))
        ev.set_response(str(d.get("response_text") or ""))
        dur = float(d.get("audio_duration") or 0.0)
        sr = int(d.get("sample_rate") or 0)
        if dur > 0 or sr > 0:
            ev.set_audio_metadata(1, sr, bool(d.get("wake_word_detected")))
            if dur > 0:
                ev.audio_duration = dur
        try:
            await asyncio.to_thread(self.store.insert, ev)
        except Exception as e:
            log.error("failed to create voice event (relay %s): %s", relay, e)
            return http_error("Failed to create voice event", 500)
        return go_json_response(event_struct(ev), 201)

    async def get_voice_event(self, uuid: str) -> web.Response:
        try:
            ev = await asyncio.to_thread(self.store.get_by_uuid, uuid)
        except NotFound:
            return http_error("Voice event not found", 404)
        except Exception as e:
            log.error("failed to get voice event %s: %s", uuid, e)
            return http_error("Internal server error", 500)
        return go_json_response(event_struct(ev))
