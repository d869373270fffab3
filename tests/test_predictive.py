"""Predictive subsystem (C25-C29); tables follow ``predictive_response_test.go``."""
import asyncio

import pytest

from loqa_hub_amd.llm.commands import Command
from loqa_hub_amd.predictive import (HYBRID, PREDICTIVE_ONLY, STREAMING_ONLY,
                                     AsyncExecutionPipeline, CommandClassifier,
                                     DeviceReliabilityTracker, NullSkillManager,
                                     PredictiveResponseEngine, SkillManagerAdapter, StatusManager,
                                     StatusUpdate, StreamingPredictiveBridge)
from loqa_hub_amd.predictive.classifier import (extract_intent_category, extract_operation_type,
                                                extract_target_id)
from loqa_hub_amd.predictive.status_manager import categorize_error
from loqa_hub_amd.predictive.types import CommandClassification
from loqa_hub_amd.skills.interfaces import SkillResponse
from loqa_hub_amd.streaming.parser import StreamingCommandParser


class MockSkillManager:
    def __init__(self, find=True, succeed=True, delay=0.0, message="done", fail_times=0):
        self.find, self.succeed, self.delay, self.message = find, succeed, delay, message
        self.fail_times, self.calls = fail_times, 0

    def find_skill_for_intent(self, intent):
        if not self.find:
            raise LookupError("no skill")
        return object()

    async def execute_skill(self, skill, intent):
        self.calls += 1
        await asyncio.sleep(self.delay)
        if self.calls <= self.fail_times:
            return SkillResponse(success=False, error="flaky")
        return SkillResponse(success=self.succeed, message=self.message,
                             error="" if self.succeed else "device offline")


def test_reliability_tracker():
    t = DeviceReliabilityTracker()
    assert t.get_reliability_score("bedroom_lights") == 0.5
    for ok in [True] * 8 + [False] * 2:
        t.update_stats("bedroom_lights", ok, 1.0)
    assert t.get_reliability_score("bedroom_lights") == pytest.approx(0.8)
    assert t.get_reliability_score("unknown_device") == 0.5


@pytest.mark.parametrize("text,cat,op", [
    ("turn off the bedroom lights", "smart_home", "control"),
    ("open the garage door", "smart_home", "control"),
    ("check if the front door is locked", "smart_home", "query"),
    ("what's the weather", "weather", "query"),
    ("play some music", "entertainment", "control"),
    ("restart the system", "system", "maintenance"),
    ("restart the router", "navigation", "maintenance"),
    ("arm the alarm", "smart_home", "critical")])
def test_classification_tables(text, cat, op):
    assert extract_intent_category(text, {}) == cat
    assert extract_operation_type(text) == op


def test_target_and_response_types():
    assert extract_target_id({"location": "kitchen", "device": "lights"}) == "device_kitchen_lights"
    assert extract_target_id({"topic": "news"}) == "topic_news"
    assert extract_target_id({}) == "general_request"
    c = CommandClassifier()
    cases = [(0.95, 0.90, 1.0, "control", "optimistic"), (0.70, 0.60, 2.0, "control", "cautious"),
             (0.95, 0.90, 15.0, "control", "progress"), (0.95, 0.90, 1.0, "critical", "confirm")]
    for conf, rel, t, op, exp in cases:
        assert c.determine_response_type(conf, rel, t, op) == exp
    assert c.estimated_execution_time("smart_home", "sequence") == 6.0
    c.update_intent_timing("smart_home", 1.0)
    assert c.get_intent_timings()["smart_home"] == pytest.approx(2.4)


def test_classify_parsed_uses_reliability():
    rel = DeviceReliabilityTracker()
    c = CommandClassifier(None, rel)
    cmd = Command("turn_off", {"location": "bedroom", "device": "light"}, 0.97, "ok")
    assert c.classify_parsed(cmd).response_type == "cautious"  # unknown device: 0.5
    for _ in range(5):
        rel.update_stats("bedroom_light", True, 0.1)
    cl = c.classify_parsed(cmd)
    # category is keyed on the intent string (reference behaviour): turn_off -> general
    assert cl.response_type == "optimistic" and cl.category == "general"
    assert cl.update_strategy == "error_only"
    light = c.classify_parsed(Command("light_off", {"location": "bedroom", "device": "light"},
                                      0.97, "ok"))
    assert light.category == "smart_home" and light.update_strategy == "silent"


def _cls(intent="turn_off", conf=0.95, rtype="optimistic", strategy="verbose"):
    return CommandClassification(intent, {"location": "bedroom", "device": "lights"}, conf, 0.92,
                                 2.0, rtype, strategy)


def test_predictive_engine_ack_and_status():
    async def go():
        eng = PredictiveResponseEngine(MockSkillManager(delay=0.01))
        resp = await eng.process_command("turn off the bedroom lights", classification=_cls())
        assert resp.immediate_ack == "Turning off the bedroom lights now"
        assert resp.execution_id.startswith("exec_")
        upd = await asyncio.wait_for(resp.status_updates.get(), 1.0)
        assert upd.type == "success" and upd.success
        await resp.done.wait()
        assert resp.success and eng.get_active_executions() == {}
        assert eng.reliability.get_reliability_score("bedroom_lights") == 1.0
        bad = PredictiveResponseEngine(MockSkillManager(find=False))
        r2 = await bad.process_command("x", classification=_cls(rtype="cautious"))
        assert r2.immediate_ack == "I'll try to turn off the bedroom lights"
        u = await asyncio.wait_for(r2.status_updates.get(), 1.0)
        assert u.type == "error" and u.message == "Sorry, I couldn't reach the bedroom lights"
        assert "no skill found" in u.error
        # silent strategy: no success update
        r3 = await eng.process_command("x", classification=_cls(strategy="silent"))
        await r3.done.wait()
        assert r3.status_updates.empty()
        confirm = eng.generate_predictive_response(_cls(rtype="confirm"))
        assert confirm.immediate_ack == "Are you sure you want to turn off the bedroom lights?"
    asyncio.run(go())


def test_async_execution_pipeline():
    async def go():
        sm = MockSkillManager(fail_times=1)
        p = AsyncExecutionPipeline(sm, retry_delay=0.01)
        q = asyncio.Queue(10)
        from loqa_hub_amd.skills.interfaces import VoiceIntent
        intent = VoiceIntent(intent="turn_on", entities={"location": "kitchen", "device": "fan"})
        p.submit_execution("e1", intent, _cls(strategy="verbose"), q)
        progress = await asyncio.wait_for(q.get(), 1.0)
        assert progress.type == "progress" and progress.message == "Retrying operation (attempt 2)"
        done = await asyncio.wait_for(q.get(), 1.0)
        assert done.type == "success" and done.message == "done"
        m = p.get_metrics()
        assert m.successful_executions == 1 and m.retried_executions == 1
        # permanent failure -> error message from entities after 2 retries
        p2 = AsyncExecutionPipeline(MockSkillManager(succeed=False), retry_delay=0.0)
        q2 = asyncio.Queue(10)
        p2.submit_execution("e2", intent, _cls(strategy="error_only"), q2)
        msgs = [await asyncio.wait_for(q2.get(), 1.0) for _ in range(3)]
        assert msgs[-1].type == "error"
        assert msgs[-1].message == "Sorry, I couldn't reach the kitchen fan"
        assert "after 2 retries" in msgs[-1].error
        # full queue is rejected without blocking
        p3 = AsyncExecutionPipeline(MockSkillManager(delay=0.2), max_concurrency=1, queue_size=1)
        p3.submit_execution("a", intent, _cls(), asyncio.Queue(10))
        await asyncio.sleep(0.01)
        p3.submit_execution("b", intent, _cls(), asyncio.Queue(10))
        with pytest.raises(RuntimeError, match="queue is full"):
            p3.submit_execution("c", intent, _cls(), asyncio.Queue(10))
        for x in (p, p2, p3):
            await x.shutdown()
    asyncio.run(go())


def test_status_manager_filtering_and_patterns():
    async def go():
        sm = StatusManager()
        q = asyncio.Queue(50)
        sm.register_execution("x", "error_only", "bedroom_lights", q)
        await sm.process_status_update(StatusUpdate("success", "ok", True, "x"))
        assert q.empty() and sm.get_metrics().silent_updates == 1
        for _ in range(3):
            await sm.process_status_update(StatusUpdate("error", "fail", False, "x",
                                                        error="connection refused"))
        await asyncio.sleep(0.01)
        msgs = []
        while not q.empty():
            msgs.append(q.get_nowait().message)
        # the pattern is recorded before enrichment (reference order), so even the
        # first error carries the suffix
        assert msgs[0] == msgs[1] == "fail - this device has been having issues"
        assert "Recovered from connection issue, retrying operation" in msgs
        p = sm.get_error_patterns()["bedroom_lights_connection"]
        assert p.occurrence_count == 3 and p.resolved
        with pytest.raises(KeyError):
            await sm.process_status_update(StatusUpdate("error", "", False, "nope"))
        assert categorize_error("request timeout") == "timeout"
        assert categorize_error("device not found") == "unavailable"
        assert categorize_error("") == "unknown"
    asyncio.run(go())


def test_bridge_strategies():
    async def go():
        rel = DeviceReliabilityTracker()
        for _ in range(3):
            rel.update_stats("bedroom_lights", True, 0.1)
        clf = CommandClassifier(None, rel)
        eng = PredictiveResponseEngine(MockSkillManager(), clf)
        fb_parser = StreamingCommandParser(None, None, enabled=False)

        class FB:
            async def parse_command(self, t):
                return Command("question", {}, 0.9, "It is sunny.")
        fb_parser.fallback = FB()
        bridge = StreamingPredictiveBridge(fb_parser, eng, StatusManager(), clf)
        s1 = await bridge.process_voice_command(
            "turn off the bedroom lights",
            parsed=Command("turn_off", {"location": "bedroom", "device": "lights"}, 0.97, "ok"))
        assert s1.strategy == PREDICTIVE_ONLY
        assert s1.predictive_response.immediate_ack == "Turning off the bedroom lights now"
        s2 = await bridge.process_voice_command(
            "play music", parsed=Command("play", {"device": "music"}, 0.85, "ok"))
        assert s2.strategy == HYBRID
        first = await asyncio.wait_for(s2.status_updates.get(), 1.0)
        assert first.message.startswith("Processing: ")
        s3 = await bridge.process_voice_command(
            "what time is it", parsed=Command("what_time", {}, 0.9, "noon"))
        assert s3.strategy == STREAMING_ONLY
        s4 = await bridge.process_voice_command("no parse available")  # classify fails
        assert s4.streaming_result is not None
        for s in (s1, s2, s3, s4):
            await asyncio.wait_for(s.task, 2.0)
        m = bridge.get_metrics()
        assert (m.predictive_only_sessions, m.hybrid_sessions, m.streaming_only_sessions,
                m.fallback_to_streaming) == (1, 1, 1, 1)
        assert m.successful_predictions == 2 and bridge.get_active_sessions() == {}
    asyncio.run(go())


def test_skill_adapter_with_manager(tmp_path):
    from loqa_hub_amd.skills import DefaultSkillLoader, SkillManager, SkillManagerConfig
    from loqa_hub_amd.skills.builtin.lights import LightsSkill
    from loqa_hub_amd.skills.interfaces import VoiceIntent

    async def go():
        mgr = SkillManager(SkillManagerConfig(skills_dir=str(tmp_path)),
                           DefaultSkillLoader(str(tmp_path)))
        await mgr.register_plugin(LightsSkill())
        ad = SkillManagerAdapter(mgr)
        intent = VoiceIntent(transcript="turn on the kitchen lights")
        r = await ad.execute_skill(ad.find_skill_for_intent(intent), intent)
        assert r.success and mgr.get_skill("builtin.lights").status.usage_count == 1
        with pytest.raises(LookupError):
            NullSkillManager().find_skill_for_intent(intent)
    asyncio.run(go())
