"""Session registry + graceful interrupt (``internal/llm/streaming_interrupt_handler.go``).

Interrupt = cancel the streaming result, drain its channels and cancel the audio
pipeline within ``grace_period``, else force-terminate (cancel the session
context) (:93-191). ``interrupt_all_sessions`` fans out in parallel
(:122-145). Reasons: user_request, new_command, timeout, error, shutdown.
"""
from __future__ import annotations

import asyncio
import time
from dataclasses import dataclass

REASON_USER_REQUEST = "user_request"
REASON_NEW_COMMAND = "new_command"
REASON_TIMEOUT = "timeout"
REASON_ERROR = "error"
REASON_SHUTDOWN = "shutdown"


@dataclass
class StreamingSession:
    id: str
    cancel: object = None            # callable: cancels the session's work
    streaming_result: object = None  # parser.StreamingResult
    audio_pipeline: object = None    # audio_pipeline.PipelineContext
    created_at: float = 0.0
    interrupted_at: float | None = None
    interrupt_reason: str = ""
    cleanup_completed: bool = False


@dataclass
class SessionMetrics:
    active_sessions: int = 0
    interrupted_count: int = 0
    average_duration_s: float = 0.0
    interrupt_reasons: dict | None = None


class StreamingInterruptHandler:
    def __init__(self, grace_period: float = 0.5, force_timeout: float = 1.0):
        self.grace_period = grace_period
        self.force_timeout = force_timeout
        self.active: dict[str, StreamingSession] = {}
        self._tasks: set[asyncio.Task] = set()

    def register_session(self, session_id: str, cancel=None, streaming_result=None,
                         audio_pipeline=None) -> StreamingSession:
        s = self.active.get(session_id)
        if s is None:
            s = StreamingSession(session_id, cancel, streaming_result, audio_pipeline,
                                 time.monotonic())
            self.active[session_id] = s
        else:  # update (the reference re-registers to attach the result)
            s.cancel = cancel or s.cancel
            s.streaming_result = streaming_result or s.streaming_result
            s.audio_pipeline = audio_pipeline or s.audio_pipeline
        return s

    def interrupt_session(self, session_id: str, reason: str) -> asyncio.Task | None:
        s = self.active.get(session_id)
        if s is None or s.interrupted_at is not None:
            return None
        s.interrupted_at = time.monotonic()
        s.interrupt_reason = reason
        t = asyncio.get_running_loop().create_task(self._graceful_shutdown(s))
        self._tasks.add(t)
        t.add_done_callback(self._tasks.discard)
        return t

    async def interrupt_all_sessions(self, reason: str) -> None:
        ts = [self.interrupt_session(sid, reason) for sid in list(self.active)]
        await asyncio.gather(*[t for t in ts if t is not None], return_exceptions=True)

    async def _graceful_shutdown(self, s: StreamingSession) -> None:
        res = s.streaming_result
        if res is not None:
            res.cancel()

        async def graceful():
            if res is not None:
                await self._drain(res)
            if s.audio_pipeline is not None:
                s.audio_pipeline.cancel()
        try:
            await asyncio.wait_for(graceful(), self.grace_period)
        except asyncio.TimeoutError:
            self._force_termination(s)
        s.cleanup_completed = True
        self.active.pop(s.id, None)

    def _force_termination(self, s: StreamingSession) -> None:
        if callable(s.cancel):
            s.cancel()
        if s.streaming_result is not None:
            s.streaming_result.close_outputs()

    async def _drain(self, res) -> None:
        deadline = time.monotonic() + self.force_timeout
        while time.monotonic() < deadline:
            progressed = False
            for ch in (res.token_stream, res.visual_tokens, res.audio_phrases):
                _, ok = ch.try_get()
                progressed |= ok
            _, fin = res.final_command.try_get()
            _, err = res.errors.try_get()
            if fin or err or not progressed:
                return

    def get_active_session_ids(self) -> list[str]:
        return list(self.active)

    def get_session_info(self, session_id: str) -> dict | None:
        s = self.active.get(session_id)
        if s is None:
            return None
        end = s.interrupted_at if s.interrupted_at is not None else time.monotonic()
        return {"id": s.id, "duration_s": end - s.created_at,
                "is_interrupted": s.interrupted_at is not None,
                "interrupt_reason": s.interrupt_reason, "cleanup_completed": s.cleanup_completed}

    def get_session_metrics(self) -> SessionMetrics:
        m = SessionMetrics(active_sessions=len(self.active), interrupt_reasons={})
        total, now = 0.0, time.monotonic()
        for s in self.active.values():
            if s.interrupted_at is not None:
                m.interrupted_count += 1
                m.interrupt_reasons[s.interrupt_reason] = m.interrupt_reasons.get(
                    s.interrupt_reason, 0) + 1
                total += s.interrupted_at - s.created_at
            else:
                total += now - s.created_at
        if self.active:
            m.average_duration_s = total / len(self.active)
        return m

    async def shutdown(self) -> None:
        await self.interrupt_all_sessions(REASON_SHUTDOWN)
