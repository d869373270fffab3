"""Structured logging with the reference's field conventions.

Mirrors ``internal/logging/logger.go``: ``initialize`` reads LOG_LEVEL /
LOG_FORMAT (json -> production-style JSON lines, anything else -> console),
level parse falls back to info, errors carry a stack. Every helper tags the
line with a ``component`` field (voice_pipeline, audio_processing + relay_id +
stage, messaging, database, tts) exactly like ``LogVoiceEvent`` (:110-129),
``LogAudioProcessing`` (:132-145), ``LogNATSEvent`` (:148-161),
``LogDatabaseOperation`` (:164-177), ``LogError`` (:180-191), ``LogWarn``
(:194-200), ``LogTTSOperation`` (:203-215). User-controlled strings pass through
``sanitize_log_input`` first.
"""
from __future__ import annotations

import json
import logging
import logging.handlers
import os
import sys
import time
import traceback

from .security import sanitize_log_input

ROOT = "loqa"
_LEVELS = {"debug": logging.DEBUG, "info": logging.INFO, "warn": logging.WARNING,
           "warning": logging.WARNING, "error": logging.ERROR, "dpanic": logging.CRITICAL,
           "panic": logging.CRITICAL, "fatal": logging.CRITICAL}


class JSONFormatter(logging.Formatter):
    def format(self, rec: logging.LogRecord) -> str:
        d = {"level": rec.levelname.lower().replace("warning", "warn"), "ts": rec.created,
             "caller": f"{rec.module}.py:{rec.lineno}", "msg": rec.getMessage()}
        fields = getattr(rec, "fields", None)
        if fields:
            for k, v in fields.items():
                d[k] = v if isinstance(v, (int, float, bool, str, type(None), list, dict)) else str(v)
        if rec.exc_info:
            d["error"] = str(rec.exc_info[1])
        if rec.levelno >= logging.ERROR:
            d["stacktrace"] = "".join(traceback.format_stack(limit=8)[:-2])
        return json.dumps(d, default=str)


class ConsoleFormatter(logging.Formatter):
    def format(self, rec: logging.LogRecord) -> str:
        ts = time.strftime("%Y-%m-%dT%H:%M:%S", time.localtime(rec.created))
        base = f"{ts}\t{rec.levelname.upper()}\t{rec.module}.py:{rec.lineno}\t{rec.getMessage()}"
        fields = getattr(rec, "fields", None)
        if fields:
            base += "\t" + json.dumps(fields, default=str)
        if rec.exc_info:
            base += "\n" + self.formatException(rec.exc_info)
        return base


def initialize(level: str | None = None, fmt: str | None = None, stream=None) -> logging.Logger:
    """``logging.Initialize`` / ``InitializeWithConfig``."""
    level = level or os.environ.get("LOG_LEVEL", "info")
    fmt = fmt or os.environ.get("LOG_FORMAT", "json")
    lg = logging.getLogger(ROOT)
    for h in list(lg.handlers):
        lg.removeHandler(h)
        if isinstance(h, _DeferredHandler):
            h.listener.stop()
    h = logging.StreamHandler(stream or sys.stderr)
    h.setFormatter(JSONFormatter() if fmt == "json" else ConsoleFormatter())
    if os.environ.get("LOQA_LOG_ASYNC", "1") != "0" and stream is None:
        # formatting + the write happen on a listener thread, not on the
        # event loop that serves the relays (front-end tail latency)
        h = _DeferredHandler(h)
    lg.addHandler(h)
    lg.setLevel(_LEVELS.get(level.lower(), logging.INFO))
    lg.propagate = False
    return lg


class _DeferredHandler(logging.handlers.QueueHandler):
    """DEBUG / INFO: the record is enqueued with its message already rendered
    (so mutable args show their state at the call) and a QueueListener thread
    formats and writes it. WARNING and above are written synchronously, in the
    caller's thread: those are the lines that explain a failure, and a process
    killed by the DP watchdog or aborted by a GPU fault must not lose them in
    the queue (ERROR stack traces then also show the caller's stack)."""

    def __init__(self, target: logging.Handler):
        import queue as _q
        super().__init__(_q.SimpleQueue())
        self.target = target
        self.listener = logging.handlers.QueueListener(self.queue, target,
                                                       respect_handler_level=True)
        self.listener.start()
        import atexit
        atexit.register(self.listener.stop)

    def emit(self, record: logging.LogRecord) -> None:
        if record.levelno >= logging.WARNING:
            self.target.handle(record)
            try:
                self.target.flush()
            except Exception:  # noqa: BLE001
                pass
            return
        super().emit(record)

    def prepare(self, record: logging.LogRecord) -> logging.LogRecord:
        record.msg = record.getMessage()
        record.args = None
        if record.exc_info and not record.exc_text:
            record.exc_text = logging.Formatter().formatException(record.exc_info)
        return record


def get(name: str = "") -> logging.Logger:
    return logging.getLogger(f"{ROOT}.{name}" if name else ROOT)


def _log(level: int, msg: str, **fields) -> None:
    get().log(level, msg, extra={"fields": fields}, stacklevel=3)


def log_voice_event(event) -> None:
    _log(logging.INFO, "Voice event processed", component="voice_pipeline",
         event_uuid=event.uuid, relay_id=sanitize_log_input(event.relay_id),
         request_id=sanitize_log_input(event.request_id), intent=sanitize_log_input(event.intent),
         confidence=event.confidence, success=event.success,
         processing_time_ms=event.processing_time_ms,
         transcription=sanitize_log_input(event.transcription))


def log_audio_processing(relay_id: str, stage: str, **fields) -> None:
    _log(logging.INFO, "Audio processing", component="audio_processing",
         relay_id=sanitize_log_input(relay_id), stage=stage, **fields)


def log_audio_processing_debug(relay_id: str, stage: str, **fields) -> None:
    _log(logging.DEBUG, "Audio processing", component="audio_processing",
         relay_id=sanitize_log_input(relay_id), stage=stage, **fields)


def debug_enabled() -> bool:
    return logging.getLogger(ROOT).isEnabledFor(logging.DEBUG)


def log_nats_event(subject: str, event_type: str, **fields) -> None:
    _log(logging.INFO, "NATS event", component="messaging", subject=subject,
         event_type=event_type, **fields)


def log_database_operation(operation: str, table: str, **fields) -> None:
    _log(logging.DEBUG, "Database operation", component="database", operation=operation,
         table=table, **fields)


def log_error(err: BaseException | str, message: str, **fields) -> None:
    _log(logging.ERROR, message, error=str(err), **fields)


def log_warn(message: str, **fields) -> None:
    _log(logging.WARNING, message, **fields)


def log_tts_operation(operation: str, **fields) -> None:
    _log(logging.INFO, "TTS operation", component="tts", operation=operation, **fields)
