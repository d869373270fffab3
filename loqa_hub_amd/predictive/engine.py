"""Predictive response engine: instant acknowledgement, asynchronous execution
(``internal/llm/predictive_response.go``).

``process_command`` classifies, generates the immediate ack + execution plan
for the response type (:190-229), and starts execution in the background
(:232-281): the intent goes to the skill manager under a 30 s timeout, a status
update is emitted per update strategy (:296-346), and the device reliability
tracker is updated.

Deliberate fix: the reference's ``classifyCommand`` is a stub
returning a hard-coded bedroom-lights classification, so every ack reads
"Turning off the bedroom lights now". Here the classification comes from the
real parse (``CommandClassifier``) and the ack / plan / status texts are
rendered from the parsed intent and entities with the reference's sentence
shapes (the reference strings are what these templates produce for
``turn_off`` + ``{location: bedroom, device: lights}``).
"""
from __future__ import annotations

import asyncio
import time
from dataclasses import dataclass, field

from ..llm.commands import Command
from ..skills.interfaces import VoiceIntent
from .classifier import CommandClassifier
from .reliability import DeviceReliabilityTracker, extract_device_id
from .types import (PREDICTIVE_CAUTIOUS, PREDICTIVE_CONFIRM, PREDICTIVE_OPTIMISTIC,
                    PREDICTIVE_PROGRESS, STATUS_ERROR, STATUS_SUCCESS, UPDATE_PROGRESS,
                    UPDATE_VERBOSE, CommandClassification, StatusUpdate)

_VERBS = {"turn_on": ("turn on", "Turning on", "on"), "turn_off": ("turn off", "Turning off", "off"),
          "dim": ("dim", "Dimming", "dimmed"), "brighten": ("brighten", "Brightening", "brighter"),
          "play": ("play", "Playing", "playing"), "stop": ("stop", "Stopping", "stopped"),
          "pause": ("pause", "Pausing", "paused"), "lock": ("lock", "Locking", "locked"),
          "unlock": ("unlock", "Unlocking", "unlocked")}


def _target(entities: dict[str, str]) -> str:
    loc, dev = entities.get("location", ""), entities.get("device", "")
    if loc and dev:
        return f"the {loc} {dev}"
    if dev:
        return f"the {dev}"
    if loc:
        return f"the {loc} lights"
    return "that"


def render_ack(c: CommandClassification) -> tuple[str, str]:
    verb, ing, _ = _VERBS.get(c.intent, (c.intent.replace("_", " "),
                                         c.intent.replace("_", " ").capitalize(), "done"))
    tgt = _target(c.entities)
    if c.response_type == PREDICTIVE_OPTIMISTIC:
        return f"{ing} {tgt} now", "Executing immediately"
    if c.response_type == PREDICTIVE_CAUTIOUS:
        return f"I'll try to {verb} {tgt}", "Attempting to reach the device"
    if c.response_type == PREDICTIVE_CONFIRM:
        return f"Are you sure you want to {verb} {tgt}?", \
            "Waiting for confirmation before proceeding"
    if c.response_type == PREDICTIVE_PROGRESS:
        return f"Starting {verb} {tgt}", \
            f"This may take about {max(1, round(c.execution_time))} seconds to complete"
    return "Processing your request", "Working on it"


def render_status(c: CommandClassification, success: bool) -> str:
    _, _, state = _VERBS.get(c.intent, ("", "", "done"))
    tgt = _target(c.entities)
    if success:
        t = tgt[0].upper() + tgt[1:] if tgt != "that" else "That"
        return f"{t} {'are' if tgt.endswith('s') else 'is'} {state}"
    return f"Sorry, I couldn't reach {tgt}"


@dataclass
class PredictiveResponse:
    immediate_ack: str
    execution_plan: str
    confidence_level: float
    update_strategy: str
    execution_id: str
    success: bool = False
    status_updates: asyncio.Queue = field(default_factory=lambda: asyncio.Queue(10))
    done: asyncio.Event = field(default_factory=asyncio.Event)

    def to_json(self) -> dict:
        return {"immediate_ack": self.immediate_ack, "execution_plan": self.execution_plan,
                "confidence_level": self.confidence_level,
                "update_strategy": self.update_strategy, "execution_id": self.execution_id}


@dataclass
class ExecutionContext:
    id: str
    intent: VoiceIntent | None
    start_time: float
    classification: CommandClassification
    response: PredictiveResponse | None = None
    task: asyncio.Task | None = None


_exec_seq = 0


def generate_execution_id() -> str:
    global _exec_seq
    _exec_seq += 1
    return f"exec_{time.time_ns()}_{_exec_seq}"


class PredictiveResponseEngine:
    def __init__(self, skill_manager, classifier: CommandClassifier | None = None,
                 reliability: DeviceReliabilityTracker | None = None):
        self.skill_manager = skill_manager
        self.reliability = reliability or (classifier.reliability if classifier else
                                           DeviceReliabilityTracker())
        self.classifier = classifier or CommandClassifier(None, self.reliability)
        self.confidence_threshold = 0.8
        self.execution_timeout = 30.0
        self.active: dict[str, ExecutionContext] = {}

    async def process_command(self, transcript: str, parsed: Command | None = None,
                              classification: CommandClassification | None = None
                              ) -> PredictiveResponse:
        if classification is None:
            classification = (self.classifier.classify_parsed(parsed) if parsed is not None
                              else await self.classifier.classify_command(transcript))
        resp = self.generate_predictive_response(classification)
        ctx = ExecutionContext(resp.execution_id, None, time.monotonic(), classification, resp)
        self.active[resp.execution_id] = ctx
        ctx.task = asyncio.get_running_loop().create_task(
            self._execute_async(ctx, transcript))
        return resp

    def generate_predictive_response(self, c: CommandClassification) -> PredictiveResponse:
        ack, plan = render_ack(c)
        return PredictiveResponse(ack, plan, c.confidence, c.update_strategy,
                                  generate_execution_id())

    async def _execute_async(self, ctx: ExecutionContext, transcript: str) -> None:
        c, resp = ctx.classification, ctx.response
        intent = VoiceIntent(id=resp.execution_id, transcript=transcript, intent=c.intent,
                             confidence=c.confidence, entities=dict(c.entities))
        ctx.intent = intent
        t0 = time.monotonic()
        skill_resp, err = None, None
        try:
            skill = self.skill_manager.find_skill_for_intent(intent)
            skill_resp = await asyncio.wait_for(self.skill_manager.execute_skill(skill, intent),
                                                self.execution_timeout)
        except Exception as e:  # noqa: BLE001
            err = e if not isinstance(e, asyncio.TimeoutError) else TimeoutError("timeout")
        self._send_status(ctx, skill_resp, err)
        resp.success = err is None and skill_resp is not None and skill_resp.success
        self.reliability.update_stats(extract_device_id(c.entities), resp.success,
                                      time.monotonic() - t0)
        self.active.pop(resp.execution_id, None)
        resp.done.set()

    def _send_status(self, ctx: ExecutionContext, skill_resp, err) -> None:
        resp, c = ctx.response, ctx.classification
        if err is not None:
            upd = StatusUpdate(STATUS_ERROR, render_status(c, False), False, resp.execution_id,
                               error=str(err) if not isinstance(err, LookupError) else
                               f"no skill found for intent: {err}")
        elif skill_resp.success:
            if resp.update_strategy not in (UPDATE_VERBOSE, UPDATE_PROGRESS):
                return
            upd = StatusUpdate(STATUS_SUCCESS, skill_resp.speech_text or render_status(c, True),
                               True, resp.execution_id)
        else:
            upd = StatusUpdate(STATUS_ERROR, "The device didn't respond as expected", False,
                               resp.execution_id, error=skill_resp.error)
        try:
            resp.status_updates.put_nowait(upd)
        except asyncio.QueueFull:
            pass

    def get_active_executions(self) -> dict[str, ExecutionContext]:
        return dict(self.active)
