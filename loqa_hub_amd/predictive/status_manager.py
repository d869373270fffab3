"""Status-update filtering, error-pattern detection and spoken updates
(``internal/llm/status_manager.go``).

* ``should_send_update`` per strategy/priority (:198-225);
* error patterns keyed ``<device>_<category>``; >= 3 occurrences trigger a
  recovery attempt (retry/reset succeed, skip/escalate do not - simulated as in
  the reference, :228-384);
* message enrichment ("(taking longer than usual)" after 5 s of silence,
  "- this device has been having issues" within the 5 min cooldown);
* spoken updates through TTS (``af_bella``, 1.1x, mp3) for errors, critical
  successes and high-priority progress; history capped at 50 per execution.

Deliberate fix: the reference compares priorities as strings
(``Priority >= PriorityHigh`` is lexicographic, so "low"/"normal" pass and
"critical" fails); here priorities are ordered low < normal < high < critical.
"""
from __future__ import annotations

import asyncio
import time
from dataclasses import dataclass, field

from ..llm.tts import TTSOptions
from .types import (STATUS_ERROR, STATUS_PROGRESS, STATUS_SUCCESS, UPDATE_ERROR_ONLY,
                    UPDATE_PROGRESS, UPDATE_SILENT, UPDATE_VERBOSE, StatusUpdate)

PRIORITY_LOW, PRIORITY_NORMAL, PRIORITY_HIGH, PRIORITY_CRITICAL = "low", "normal", "high", "critical"
_RANK = {PRIORITY_LOW: 0, PRIORITY_NORMAL: 1, PRIORITY_HIGH: 2, PRIORITY_CRITICAL: 3}

RECOVERY_RETRY, RECOVERY_RESET, RECOVERY_FALLBACK = "retry", "reset", "fallback"
RECOVERY_SKIP, RECOVERY_ESCALATE = "skip", "escalate"


@dataclass
class StatusContext:
    execution_id: str
    update_strategy: str
    device_id: str
    updates: asyncio.Queue
    last_update: float = field(default_factory=time.monotonic)
    audio_enabled: bool = True
    priority: str = PRIORITY_NORMAL
    error_count: int = 0
    success_count: int = 0


@dataclass
class RecoveryAction:
    type: str
    description: str
    delay: float
    max_retries: int
    success: bool = False


@dataclass
class ErrorPattern:
    device_id: str
    error_type: str
    occurrence_count: int = 1
    last_occurrence: float = field(default_factory=time.monotonic)
    recovery_actions: list[RecoveryAction] = field(default_factory=list)
    resolved: bool = False


@dataclass
class StatusMetrics:
    total_updates: int = 0
    successful_updates: int = 0
    failed_updates: int = 0
    audio_updates: int = 0
    silent_updates: int = 0
    error_recoveries: int = 0
    average_update_latency: float = 0.0
    error_patterns_detected: int = 0
    recovery_success_rate: float = 0.0


def determine_priority(strategy: str) -> str:
    return {UPDATE_SILENT: PRIORITY_LOW, UPDATE_ERROR_ONLY: PRIORITY_NORMAL,
            UPDATE_VERBOSE: PRIORITY_HIGH, UPDATE_PROGRESS: PRIORITY_HIGH}.get(strategy,
                                                                              PRIORITY_NORMAL)


def categorize_error(msg: str) -> str:
    if not msg:
        return "unknown"
    m = msg.lower()
    if "timeout" in m or "no response" in m:
        return "timeout"
    if "connection" in m or "network" in m:
        return "connection"
    if "permission" in m or "unauthorized" in m:
        return "permission"
    if "not found" in m or "unavailable" in m:
        return "unavailable"
    if "invalid" in m or "bad request" in m:
        return "invalid_request"
    return "generic"


def should_send_update(ctx: StatusContext, u: StatusUpdate) -> bool:
    s = ctx.update_strategy
    if s == UPDATE_SILENT:
        return u.type == STATUS_ERROR and ctx.priority == PRIORITY_CRITICAL
    if s == UPDATE_ERROR_ONLY:
        return u.type == STATUS_ERROR or (u.type == STATUS_SUCCESS and
                                          ctx.priority == PRIORITY_CRITICAL)
    if s == UPDATE_VERBOSE:
        return True
    if s == UPDATE_PROGRESS:
        return u.type in (STATUS_PROGRESS, STATUS_ERROR, STATUS_SUCCESS)
    return u.type == STATUS_ERROR


class StatusManager:
    def __init__(self, tts=None):
        self.tts = tts
        self.active: dict[str, StatusContext] = {}
        self.history: dict[str, list[StatusUpdate]] = {}
        self.patterns: dict[str, ErrorPattern] = {}
        self.max_history = 50
        self.error_cooldown = 300.0
        self.update_timeout = 10.0
        self.enable_audio = True
        self.metrics = StatusMetrics()
        self._bg: set[asyncio.Task] = set()

    def register_execution(self, execution_id: str, strategy: str, device_id: str,
                           updates: asyncio.Queue) -> None:
        self.active[execution_id] = StatusContext(execution_id, strategy, device_id, updates,
                                                  audio_enabled=self.enable_audio,
                                                  priority=determine_priority(strategy))
        self.history[execution_id] = []

    def unregister_execution(self, execution_id: str) -> None:
        self.active.pop(execution_id, None)
        h = self.history.get(execution_id)
        if h is not None and len(h) > 10:
            self.history[execution_id] = h[-10:]

    async def process_status_update(self, u: StatusUpdate) -> None:
        t0 = time.monotonic()
        ctx = self.active.get(u.execution_id)
        if ctx is None:
            raise KeyError(f"no active status context for execution {u.execution_id}")
        if not should_send_update(ctx, u):
            self._metrics(True, time.monotonic() - t0, True)
            return
        if u.type == STATUS_ERROR:
            self._handle_error_pattern(ctx, u)
        self._enhance(ctx, u)
        err = None
        try:
            await self._send(ctx, u)
        except Exception as e:  # noqa: BLE001
            err = e
        h = self.history.setdefault(u.execution_id, [])
        h.append(u)
        if len(h) > self.max_history:
            del h[:-self.max_history]
        self._metrics(err is None, time.monotonic() - t0, False)
        if err is not None:
            raise err

    def _handle_error_pattern(self, ctx: StatusContext, u: StatusUpdate) -> None:
        et = categorize_error(u.error)
        key = f"{ctx.device_id}_{et}"
        p = self.patterns.get(key)
        if p is None:
            p = self.patterns[key] = ErrorPattern(ctx.device_id, et)
        else:
            p.occurrence_count += 1
            p.last_occurrence = time.monotonic()
        if p.occurrence_count >= 3 and not p.resolved:
            self.metrics.error_patterns_detected += 1
            t = asyncio.get_running_loop().create_task(self._recover(ctx, p))
            self._bg.add(t)
            t.add_done_callback(self._bg.discard)

    async def _recover(self, ctx: StatusContext, p: ErrorPattern) -> None:
        a = {"timeout": RecoveryAction(RECOVERY_RETRY, "Retrying with extended timeout", 3.0, 2),
             "connection": RecoveryAction(RECOVERY_RESET, "Resetting device connection", 5.0, 1),
             "unavailable": RecoveryAction(RECOVERY_SKIP, "Device temporarily unavailable", 0, 0)
             }.get(p.error_type, RecoveryAction(RECOVERY_ESCALATE,
                                                "Error requires manual attention", 0, 0))
        a.success = a.type in (RECOVERY_RETRY, RECOVERY_RESET)
        p.recovery_actions.append(a)
        p.resolved = a.success
        self.metrics.error_recoveries += 1
        if a.success:
            self.metrics.recovery_success_rate = (self.metrics.recovery_success_rate + 1.0) / 2
        msg = (f"Recovered from {p.error_type} issue, retrying operation" if a.success else
               f"Could not recover from {p.error_type} issue automatically")
        try:
            await self._send(ctx, StatusUpdate(STATUS_PROGRESS, msg, False, ctx.execution_id))
        except Exception:  # noqa: BLE001
            pass

    def _enhance(self, ctx: StatusContext, u: StatusUpdate) -> None:
        if u.type == STATUS_PROGRESS and time.monotonic() - ctx.last_update > 5.0:
            u.message = f"{u.message} (taking longer than usual)"
        if u.type == STATUS_ERROR and self.has_recent_errors(ctx.device_id):
            u.message = f"{u.message} - this device has been having issues"

    async def _send(self, ctx: StatusContext, u: StatusUpdate) -> None:
        try:
            await asyncio.wait_for(ctx.updates.put(u), self.update_timeout)
        except asyncio.TimeoutError:
            raise TimeoutError("timeout sending status update") from None
        if ctx.audio_enabled and self._should_speak(ctx, u) and self.tts is not None:
            t = asyncio.get_running_loop().create_task(self._speak(u))
            self._bg.add(t)
            t.add_done_callback(self._bg.discard)
        ctx.last_update = time.monotonic()

    @staticmethod
    def _should_speak(ctx: StatusContext, u: StatusUpdate) -> bool:
        if u.type == STATUS_ERROR:
            return True
        if u.type == STATUS_SUCCESS:
            return ctx.priority == PRIORITY_CRITICAL
        if u.type == STATUS_PROGRESS:
            return _RANK[ctx.priority] >= _RANK[PRIORITY_HIGH]
        return False

    async def _speak(self, u: StatusUpdate) -> None:
        try:
            await self.tts.synthesize(u.message, TTSOptions("af_bella", 1.1, "mp3", True))
            self.metrics.audio_updates += 1
        except Exception:  # noqa: BLE001
            pass

    def has_recent_errors(self, device_id: str) -> bool:
        now = time.monotonic()
        return any(p.device_id == device_id and now - p.last_occurrence < self.error_cooldown
                   for p in self.patterns.values())

    def _metrics(self, ok: bool, latency: float, silent: bool) -> None:
        m = self.metrics
        m.total_updates += 1
        if ok:
            m.successful_updates += 1
        else:
            m.failed_updates += 1
        if silent:
            m.silent_updates += 1
        m.average_update_latency = latency if m.total_updates == 1 else \
            (m.average_update_latency + latency) / 2

    def get_metrics(self) -> StatusMetrics:
        return StatusMetrics(**vars(self.metrics))

    def get_error_patterns(self) -> dict[str, ErrorPattern]:
        return dict(self.patterns)
