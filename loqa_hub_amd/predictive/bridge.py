"""Streaming-predictive bridge: the primary processing engine
(``internal/llm/streaming_predictive_bridge.go``).

``process_voice_command``: classify, then choose a strategy (:186-206):
``predictive_only`` (confidence >= 0.95 and optimistic), ``streaming_only``
(intent mentions what/how/explain, or confidence below 0.8) or ``hybrid``.
Hybrid/predictive register with the status manager, start the predictive
engine and monitor its status updates (30 s timeout); hybrid also emits a
"Processing: <ack>" visual update; streaming-only starts the streaming parse.
Classification failures fall back to streaming-only.

MI355X-first differences:
* the classification comes from an already-parsed command when the caller has
  one (the constrained GPU decode), so the bridge adds no LLM pass; with
  ``streamed`` (that decode's streaming result) the streaming-only strategy
  monitors it instead of starting a second, streaming parse;
* streaming-only sessions monitor the real streaming result (completion or
  error) instead of simulating a 10 s completion (:345-436).
"""
from __future__ import annotations

import asyncio
import time
from dataclasses import dataclass, field

from ..llm.commands import Command
from .engine import PredictiveResponse, PredictiveResponseEngine
from .reliability import extract_device_id
from .status_manager import StatusManager
from .types import PREDICTIVE_OPTIMISTIC, STATUS_PROGRESS, CommandClassification, StatusUpdate

HYBRID, PREDICTIVE_ONLY, STREAMING_ONLY = "hybrid", "predictive_only", "streaming_only"


@dataclass
class BridgeSession:
    session_id: str
    user_transcript: str
    start_time: float = field(default_factory=time.monotonic)
    classification: CommandClassification | None = None
    predictive_response: PredictiveResponse | None = None
    streaming_result: object = None
    strategy: str = ""
    status_updates: asyncio.Queue = field(default_factory=lambda: asyncio.Queue(20))
    first_token_time: float = 0.0
    prediction_time: float = 0.0
    streaming_active: bool = False
    prediction_active: bool = False
    completed: bool = False
    task: asyncio.Task | None = None


@dataclass
class BridgeMetrics:
    total_sessions: int = 0
    streaming_only_sessions: int = 0
    predictive_only_sessions: int = 0
    hybrid_sessions: int = 0
    average_response_time: float = 0.0
    average_prediction_time: float = 0.0
    successful_predictions: int = 0
    failed_predictions: int = 0
    fallback_to_streaming: int = 0
    user_interruptions: int = 0


_seq = 0


def generate_session_id() -> str:
    global _seq
    _seq += 1
    return f"session_{time.time_ns()}_{_seq}"


class StreamingPredictiveBridge:
    MONITOR_TIMEOUT = 30.0

    def __init__(self, streaming_parser, engine: PredictiveResponseEngine,
                 status_manager: StatusManager, classifier=None, execution_pipeline=None):
        self.streaming_parser = streaming_parser
        self.engine = engine
        self.status_manager = status_manager
        self.classifier = classifier or engine.classifier
        self.execution_pipeline = execution_pipeline
        self.confidence_threshold = 0.8
        self.active: dict[str, BridgeSession] = {}
        self.metrics = BridgeMetrics()

    async def process_voice_command(self, transcript: str, parsed: Command | None = None,
                                    streamed=None) -> BridgeSession:
        s = BridgeSession(generate_session_id(), transcript)
        s.streaming_result = streamed
        self.active[s.session_id] = s
        try:
            s.classification = (self.classifier.classify_parsed(parsed) if parsed is not None
                                else await self.classifier.classify_command(transcript))
        except Exception:  # noqa: BLE001
            return await self._streaming_only(s, fallback=True)
        s.prediction_time = time.monotonic()
        s.strategy = self.determine_processing_strategy(s.classification)
        if s.strategy == STREAMING_ONLY:
            return await self._streaming_only(s)
        return await self._predictive(s, hybrid=s.strategy == HYBRID)

    def determine_processing_strategy(self, c: CommandClassification) -> str:
        if c.confidence >= 0.95 and c.response_type == PREDICTIVE_OPTIMISTIC:
            return PREDICTIVE_ONLY
        low = c.intent.lower()
        if "what" in low or "how" in low or "explain" in low:
            return STREAMING_ONLY
        if c.confidence >= self.confidence_threshold:
            return HYBRID
        return STREAMING_ONLY

    async def _predictive(self, s: BridgeSession, hybrid: bool) -> BridgeSession:
        s.prediction_active = True
        s.streaming_active = hybrid
        self.status_manager.register_execution(s.session_id, s.classification.update_strategy,
                                               extract_device_id(s.classification.entities),
                                               s.status_updates)
        try:
            s.predictive_response = await self.engine.process_command(
                s.user_transcript, classification=s.classification)
        except Exception:  # noqa: BLE001
            return await self._streaming_only(s, fallback=True)
        if hybrid:
            try:
                s.status_updates.put_nowait(StatusUpdate(
                    STATUS_PROGRESS, f"Processing: {s.predictive_response.immediate_ack}", False,
                    s.session_id))
                s.first_token_time = time.monotonic()
            except asyncio.QueueFull:
                pass
        s.task = asyncio.get_running_loop().create_task(self._monitor_predictive(s))
        self._count(HYBRID if hybrid else PREDICTIVE_ONLY)
        return s

    async def _streaming_only(self, s: BridgeSession, fallback: bool = False) -> BridgeSession:
        s.streaming_active, s.prediction_active = True, False
        try:
            if s.streaming_result is None:
                s.streaming_result = await self.streaming_parser.parse_command_streaming(
                    s.user_transcript)
        except Exception as e:
            self._cleanup(s.session_id)
            raise RuntimeError(("fallback streaming failed: " if fallback else
                                "failed to start streaming: ") + str(e)) from e
        s.first_token_time = time.monotonic()
        s.task = asyncio.get_running_loop().create_task(self._monitor_streaming(s))
        if fallback:
            self.metrics.fallback_to_streaming += 1
        else:
            self._count(STREAMING_ONLY)
        return s

    async def _monitor_predictive(self, s: BridgeSession) -> None:
        resp = s.predictive_response
        ok = False
        try:
            deadline = time.monotonic() + self.MONITOR_TIMEOUT
            while True:
                get = asyncio.ensure_future(resp.status_updates.get())
                done_w = asyncio.ensure_future(resp.done.wait())
                finished, _ = await asyncio.wait({get, done_w},
                                                 timeout=max(0.0, deadline - time.monotonic()),
                                                 return_when=asyncio.FIRST_COMPLETED)
                if get in finished:
                    done_w.cancel()
                    u = get.result()
                    u.execution_id = s.session_id
                    try:
                        await self.status_manager.process_status_update(u)
                    except Exception:  # noqa: BLE001
                        pass
                    continue
                get.cancel()
                if done_w in finished:
                    while not resp.status_updates.empty():  # flush late updates
                        u = resp.status_updates.get_nowait()
                        u.execution_id = s.session_id
                        try:
                            await self.status_manager.process_status_update(u)
                        except Exception:  # noqa: BLE001
                            pass
                    ok = resp.success
                    s.completed = True
                    break
                done_w.cancel()
                break  # timeout
        finally:
            self._completion(s, ok)
            self._cleanup(s.session_id)

    async def _monitor_streaming(self, s: BridgeSession) -> None:
        ok = False
        try:
            res = s.streaming_result
            try:
                cmd = await asyncio.wait_for(res.final_command.get(), self.MONITOR_TIMEOUT)
                ok = cmd is not None
            except Exception:  # noqa: BLE001  (closed without a command / timeout)
                ok = False
            s.completed = True
        finally:
            self._completion(s, ok)
            self._cleanup(s.session_id)

    def _count(self, strategy: str) -> None:
        m = self.metrics
        m.total_sessions += 1
        if strategy == HYBRID:
            m.hybrid_sessions += 1
        elif strategy == PREDICTIVE_ONLY:
            m.predictive_only_sessions += 1
        else:
            m.streaming_only_sessions += 1

    def _completion(self, s: BridgeSession, success: bool) -> None:
        m = self.metrics
        rt = time.monotonic() - s.start_time
        m.average_response_time = rt if m.total_sessions <= 1 else (m.average_response_time + rt) / 2
        if s.prediction_active:
            pt = s.prediction_time - s.start_time
            m.average_prediction_time = pt if m.total_sessions <= 1 else \
                (m.average_prediction_time + pt) / 2
            if success:
                m.successful_predictions += 1
            else:
                m.failed_predictions += 1

    def _cleanup(self, session_id: str) -> None:
        self.active.pop(session_id, None)
        self.status_manager.unregister_execution(session_id)

    def get_metrics(self) -> BridgeMetrics:
        return BridgeMetrics(**vars(self.metrics))

    def get_active_sessions(self) -> dict[str, BridgeSession]:
        return dict(self.active)

    def interrupt_session(self, session_id: str) -> None:
        s = self.active.get(session_id)
        if s is None:
            raise KeyError(f"session {session_id} not found")
        if s.task is not None:
            s.task.cancel()
        if s.streaming_result is not None:
            s.streaming_result.cancel()
        self.metrics.user_interruptions += 1
