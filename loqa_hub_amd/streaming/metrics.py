"""Streaming metrics collector (``internal/llm/streaming_metrics.go``).

Aggregates use the reference's pairwise running average (new = (old + x) / 2)
for first-token / first-phrase / completion latency and tokens/s; error rate =
interrupted / total sessions; quality score and recommendations (:320-399);
health: critical if error > 0.2, warning if error > 0.1 or first token > 2 s,
healthy once a session completed, else unknown (:402-416). Session history is
pruned to the last hour once more than 100 sessions are held.
Durations are exported as Go ``time.Duration`` nanoseconds so the
``/api/streaming/metrics`` JSON has the reference's shape.
"""
from __future__ import annotations

import json
import time
from dataclasses import dataclass, field

from .parser import StreamingMetrics

CRITICAL, WARNING, HEALTHY, UNKNOWN = "critical", "warning", "healthy", "unknown"
NS = 1_000_000_000


@dataclass
class AggregateMetrics:
    total_sessions: int = 0
    completed_sessions: int = 0
    interrupted_sessions: int = 0
    average_first_token: float = 0.0
    average_first_phrase: float = 0.0
    average_completion: float = 0.0
    total_tokens: int = 0
    total_phrases: int = 0
    streaming_enabled: bool = False
    fallback_usage: int = 0
    error_rate: float = 0.0
    throughput_tokens_per_sec: float = 0.0
    last_updated: float = field(default_factory=time.time)

    def to_json(self) -> dict:
        from ..events import rfc3339
        from datetime import datetime, timezone
        return {"total_sessions": self.total_sessions,
                "completed_sessions": self.completed_sessions,
                "interrupted_sessions": self.interrupted_sessions,
                "average_first_token": int(self.average_first_token * NS),
                "average_first_phrase": int(self.average_first_phrase * NS),
                "average_completion": int(self.average_completion * NS),
                "total_tokens": self.total_tokens, "total_phrases": self.total_phrases,
                "streaming_enabled": self.streaming_enabled,
                "fallback_usage": self.fallback_usage, "error_rate": self.error_rate,
                "throughput_tokens_per_sec": self.throughput_tokens_per_sec,
                "last_updated": rfc3339(datetime.fromtimestamp(self.last_updated, timezone.utc))}


def _avg(old: float, x: float) -> float:
    return x if old == 0 else (old + x) / 2


def quality_score(m: StreamingMetrics) -> float:
    s = 1.0 - 0.2 * m.interrupt_count - 0.1 * m.buffer_overflows
    if m.first_token_time:
        lat = m.first_token_time - m.start_time
        if lat < 0.5:
            s += 0.1
        elif lat > 2.0:
            s -= 0.1
    if m.completion_time:
        s += 0.1
    return min(1.0, max(0.0, s))


class StreamingMetricsCollector:
    def __init__(self, enabled: bool = True):
        self.enabled = enabled
        self.sessions: dict[str, StreamingMetrics] = {}
        self.agg = AggregateMetrics(streaming_enabled=enabled)
        self.start_time = time.monotonic()

    def record_session_start(self, session_id: str) -> None:
        if not self.enabled:
            return
        self.sessions[session_id] = StreamingMetrics(start_time=time.monotonic())
        self.agg.total_sessions += 1

    def record_fallback(self) -> None:
        self.agg.fallback_usage += 1

    def record_session_metrics(self, session_id: str, m: StreamingMetrics | None) -> None:
        if not self.enabled or m is None:
            return
        self.sessions[session_id] = m
        a = self.agg
        if m.completion_time:
            a.completed_sessions += 1
        if m.interrupt_count > 0:
            a.interrupted_sessions += 1
        if m.first_token_time:
            a.average_first_token = _avg(a.average_first_token, m.first_token_time - m.start_time)
        if m.first_phrase_time:
            a.average_first_phrase = _avg(a.average_first_phrase,
                                          m.first_phrase_time - m.start_time)
        if m.completion_time:
            a.average_completion = _avg(a.average_completion, m.completion_time - m.start_time)
        a.total_tokens += m.token_count
        a.total_phrases += m.phrase_count
        if m.completion_time and m.token_count > 0:
            d = m.completion_time - m.start_time
            if d > 0:
                a.throughput_tokens_per_sec = _avg(a.throughput_tokens_per_sec, m.token_count / d)
        if a.total_sessions > 0:
            a.error_rate = a.interrupted_sessions / a.total_sessions
        a.last_updated = time.time()
        if len(self.sessions) > 100:
            cutoff = time.monotonic() - 3600
            for sid in [s for s, x in self.sessions.items() if x.start_time < cutoff]:
                del self.sessions[sid]

    def get_aggregate_metrics(self) -> AggregateMetrics:
        if not self.enabled:
            return AggregateMetrics(streaming_enabled=False)
        return AggregateMetrics(**vars(self.agg))

    def assess_health_status(self) -> str:
        a = self.agg
        if a.error_rate > 0.2:
            return CRITICAL
        if a.error_rate > 0.1 or a.average_first_token > 2.0:
            return WARNING
        if a.completed_sessions > 0:
            return HEALTHY
        return UNKNOWN

    def recommendations(self) -> dict:
        a = self.agg
        r = {"optimal_buffer_time": 2 * NS, "optimal_concurrency": 3, "recommend_streaming": True,
             "estimated_improvement": "", "configuration_changes": None}
        changes = []
        if a.average_first_token > 1.0:
            changes.append("Consider reducing STREAMING_MAX_BUFFER_TIME to improve responsiveness")
            r["optimal_buffer_time"] = NS
        if a.error_rate > 0.1:
            changes.append("High error rate detected - consider enabling STREAMING_FALLBACK_ENABLED")
            r["recommend_streaming"] = False
        if a.throughput_tokens_per_sec < 10:
            changes.append("Low throughput - consider increasing STREAMING_AUDIO_CONCURRENCY")
            r["optimal_concurrency"] = 5
        r["configuration_changes"] = changes or None
        return r

    def recent_sessions(self) -> list[dict]:
        out = []
        cutoff = time.monotonic() - 600
        for sid, m in self.sessions.items():
            if m.start_time <= cutoff:
                continue
            total = (m.completion_time - m.start_time) if m.completion_time else 0.0
            out.append({
                "session_id": sid,
                "first_token_latency": int((m.first_token_time - m.start_time) * NS)
                if m.first_token_time else 0,
                "first_phrase_latency": int((m.first_phrase_time - m.start_time) * NS)
                if m.first_phrase_time else 0,
                "total_duration": int(total * NS), "token_count": m.token_count,
                "phrase_count": m.phrase_count, "buffer_overflows": m.buffer_overflows,
                "interrupt_count": m.interrupt_count, "was_interrupted": m.interrupt_count > 0,
                "completed_naturally": bool(m.completion_time), "error_encountered": False,
                "tokens_per_second": (m.token_count / total) if total > 0 and m.token_count else 0.0,
                "quality_score": quality_score(m)})
        return out

    def generate_performance_report(self) -> dict:
        if not self.enabled:
            return {"summary": AggregateMetrics(streaming_enabled=False).to_json(),
                    "recent_sessions": None, "performance_trends": None,
                    "recommended_settings": None, "health_status": "disabled"}
        return {"summary": self.agg.to_json(), "recent_sessions": self.recent_sessions(),
                "performance_trends": {
                    "last_hour_sessions": len(self.sessions),
                    "last_hour_avg_latency": int(self.agg.average_first_token * NS),
                    "last_hour_error_rate": self.agg.error_rate, "trend_direction": "stable",
                    "latency_trend": None, "throughput_trend": None},
                "recommended_settings": self.recommendations(),
                "health_status": self.assess_health_status()}

    def export_metrics(self) -> bytes:
        return json.dumps(self.generate_performance_report(), indent=2).encode()

    def reset(self) -> None:
        self.sessions.clear()
        self.agg = AggregateMetrics(streaming_enabled=self.enabled)
        self.start_time = time.monotonic()
