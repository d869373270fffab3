"""``/api/streaming/*`` monitoring endpoints (documented in the reference's
``API.md:325-520``; not routed by its server). Durations are rendered as Go
duration strings ("250ms", "2.1s") as in the documented examples.

GET /api/streaming/health           StreamingComponents.get_health_status()
GET /api/streaming/metrics          performance report
GET /api/streaming/sessions         active sessions + session metrics
GET /api/streaming/metrics/export   ?format=json&include_sessions=true|false
"""
from __future__ import annotations

from aiohttp import web

from ..config import format_go_duration
from .skills import write_error, write_json

NS = 1e9
_DURATION_KEYS = {"average_first_token", "average_first_phrase", "average_completion",
                  "first_token_latency", "first_phrase_latency", "total_duration",
                  "last_hour_avg_latency", "optimal_buffer_time"}


def _durations(obj):
    if isinstance(obj, dict):
        return {k: (format_go_duration(v / NS) if k in _DURATION_KEYS and isinstance(v, (int, float))
                    else _durations(v)) for k, v in obj.items()}
    if isinstance(obj, list):
        return [_durations(v) for v in obj]
    return obj


class StreamingHandler:
    def __init__(self, components):
        self.c = components

    def routes(self) -> list[web.RouteDef]:
        return [web.get("/api/streaming/health", self.health),
                web.get("/api/streaming/metrics", self.metrics),
                web.get("/api/streaming/sessions", self.sessions),
                web.get("/api/streaming/metrics/export", self.export)]

    def _unavailable(self) -> web.Response | None:
        if self.c is None:
            return write_error(503, "streaming components not initialized")
        return None

    async def health(self, req: web.Request) -> web.Response:
        return self._unavailable() or write_json(200, self.c.get_health_status().to_json())

    async def metrics(self, req: web.Request) -> web.Response:
        return self._unavailable() or write_json(
            200, _durations(self.c.metrics.generate_performance_report()))

    async def sessions(self, req: web.Request) -> web.Response:
        if self._unavailable():
            return self._unavailable()
        ih = self.c.interrupt_handler
        active = []
        for sid in ih.get_active_session_ids():
            info = ih.get_session_info(sid)
            if info is not None:
                info = dict(info)
                info["duration"] = format_go_duration(info.pop("duration_s"))
                active.append(info)
        m = ih.get_session_metrics()
        return write_json(200, {"active_sessions": active, "metrics": {
            "active_sessions": m.active_sessions, "interrupted_count": m.interrupted_count,
            "average_duration": format_go_duration(m.average_duration_s),
            "interrupt_reasons": m.interrupt_reasons or {}}})

    async def export(self, req: web.Request) -> web.Response:
        if self._unavailable():
            return self._unavailable()
        fmt = req.query.get("format", "json")
        if fmt != "json":
            return write_error(400, "unsupported export format: " + fmt)
        rep = self.c.metrics.generate_performance_report()
        if req.query.get("include_sessions", "true").lower() in ("false", "0", "f"):
            rep.pop("recent_sessions", None)
        return write_json(200, _durations(rep))
