"""Per-stage tracing (SURVEY §5.1 "New").

The reference's only timing is ad-hoc ``time.Since`` logging
(``stt_client.go:185,341``, ``openai_tts_client.go:206``,
``command_queue.go:119-121``) and ``req_<nanos>`` ids. Here every utterance
stage is a span: host stages on the monotonic clock, GPU stages bracketed by
HIP events recorded on the compute stream (so a span measures device time,
not launch time, and recording never synchronises the stream). Spans are
kept in a bounded ring and exported as

* a Chrome-trace / Perfetto JSON (``chrome_trace()``), and
* per-stage count / mean / p50 / p99 summaries (``summary()``) for
  ``/api/metrics`` and the streaming metrics endpoints.

Stages used by the pipeline: recv, arbitration, h2d, log_mel, encode,
stt_decode, llm_prefill, llm_decode, parse, queue, tts, publish.
"""
from __future__ import annotations

import collections
import contextlib
import json
import os
import threading
import time


class Span:
    __slots__ = ("name", "t0", "t1", "attrs", "ev0", "ev1", "tid")

    def __init__(self, name: str, attrs: dict, tid: int):
        self.name, self.attrs, self.tid = name, attrs, tid
        self.t0 = time.monotonic()
        self.t1 = None
        self.ev0 = self.ev1 = None

    def duration_ms(self) -> float | None:
        if self.ev1 is not None:
            if not self.ev1.query():
                return None          # device work still in flight
            return float(self.ev0.elapsed_time(self.ev1))
        return None if self.t1 is None else (self.t1 - self.t0) * 1e3


class Tracer:
    def __init__(self, capacity: int = 20000, enabled: bool | None = None):
        if enabled is None:
            enabled = os.environ.get("LOQA_TRACE", "1") != "0"
        self.enabled = enabled
        self.spans: collections.deque[Span] = collections.deque(maxlen=capacity)
        self._lock = threading.Lock()
        self._origin = time.monotonic()

    @contextlib.contextmanager
    def span(self, name: str, device=None, **attrs):
        """Host span; with ``device`` (a CUDA/HIP device or stream owner) the
        span is bracketed by events on the current stream of that device."""
        if not self.enabled:
            yield None
            return
        s = Span(name, attrs, threading.get_ident())
        if device is not None:
            import torch
            if torch.device(device).type == "cuda":
                s.ev0 = torch.cuda.Event(enable_timing=True)
                s.ev0.record()
        try:
            yield s
        finally:
            if s.ev0 is not None:
                import torch
                s.ev1 = torch.cuda.Event(enable_timing=True)
                s.ev1.record()
            s.t1 = time.monotonic()
            with self._lock:
                self.spans.append(s)

    def record(self, name: str, t0: float, t1: float, **attrs) -> None:
        """A span from two monotonic timestamps taken elsewhere."""
        if not self.enabled:
            return
        s = Span(name, attrs, threading.get_ident())
        s.t0, s.t1 = t0, t1
        with self._lock:
            self.spans.append(s)

    def summary(self) -> dict[str, dict]:
        with self._lock:
            spans = list(self.spans)
        by: dict[str, list[float]] = collections.defaultdict(list)
        for s in spans:
            d = s.duration_ms()
            if d is not None:
                by[s.name].append(d)
        out = {}
        for name, xs in by.items():
            xs.sort()
            n = len(xs)
            out[name] = {"count": n, "mean_ms": sum(xs) / n, "p50_ms": xs[n // 2],
                         "p99_ms": xs[min(n - 1, int(n * 0.99))]}
        return out

    def chrome_trace(self) -> str:
        """Chrome trace-event JSON ("X" complete events, microseconds)."""
        with self._lock:
            spans = list(self.spans)
        ev = []
        for s in spans:
            d = s.duration_ms()
            if d is None:
                continue
            ev.append({"name": s.name, "ph": "X", "pid": os.getpid(), "tid": s.tid,
                       "ts": (s.t0 - self._origin) * 1e6, "dur": d * 1e3,
                       "args": {k: str(v) for k, v in s.attrs.items()}})
        return json.dumps({"traceEvents": ev, "displayTimeUnit": "ms"})

    def clear(self) -> None:
        with self._lock:
            self.spans.clear()


_tracer = Tracer()


def tracer() -> Tracer:
    return _tracer
