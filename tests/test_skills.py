"""Skills subsystem (C32-C36) and the /api/skills surface (C11)."""
import asyncio
import json
import stat
import sys
import textwrap

import pytest
from aiohttp import web
from aiohttp.test_utils import TestClient, TestServer

from loqa_hub_amd.api.skills import SkillsHandler
from loqa_hub_amd.skills import (BuiltinExecutor, DefaultSkillLoader, InvalidManifest,
                                 NoSkillCanHandle, SkillAlreadyLoaded, SkillManager,
                                 SkillManagerConfig, SkillManifest, SkillNotFound, SkillState,
                                 VoiceIntent, default_builtin_executor)
from loqa_hub_amd.skills.builtin.lights import LightsSkill, parse_lighting
from loqa_hub_amd.skills.loader import contains_words, validate_skill_path
from loqa_hub_amd.utils import gojson

MODULE_SKILL = textwrap.dedent('''
    from loqa_hub_amd.skills.interfaces import *

    class Echo(SkillPlugin):
        def __init__(self):
            self.cfg = None
            self.status = SkillStatus(SkillState.LOADING, False)
        async def initialize(self, config):
            self.cfg = config
            self.status = SkillStatus(SkillState.READY, True)
        async def teardown(self):
            self.status.state = SkillState.SHUTDOWN
        def can_handle(self, intent):
            return "echo" in intent.transcript
        async def handle_intent(self, intent):
            if "fail" in intent.transcript:
                raise RuntimeError("boom")
            return SkillResponse(success=True, message="echo:" + intent.transcript)
        def get_manifest(self):
            return None
        def get_status(self):
            return self.status
        def get_config(self):
            return self.cfg
        async def update_config(self, config):
            self.cfg = config
        async def health_check(self):
            pass

    def new_skill():
        return Echo()
''')

PROCESS_SKILL = textwrap.dedent('''\
    #!{py}
    import json, sys
    for line in sys.stdin:
        req = json.loads(line)
        m = req["method"]
        if m == "handle_intent":
            res = {{"success": True, "message": "proc:" + req["params"]["transcript"],
                   "speech_text": "done"}}
        else:
            res = {{}}
        sys.stdout.write(json.dumps({{"id": req["id"], "result": res}}) + "\\n")
        sys.stdout.flush()
''')


def manifest(sid, mode="none", priority=1, trust="", examples=("echo this",)):
    return {"id": sid, "name": sid.title(), "version": "1.0.0", "description": "d",
            "author": "a", "license": "MIT",
            "intent_patterns": [{"name": "p", "examples": list(examples), "min_confidence": 0.5,
                                 "priority": priority, "enabled": True}],
            "languages": ["en"], "categories": ["test"], "permissions": [],
            "min_loqa_version": "0.1", "load_on_startup": True, "singleton": True,
            "timeout": "5s", "sandbox_mode": mode, "trust_level": trust}


@pytest.fixture
def skills_root(tmp_path):
    root = tmp_path / "skills"
    root.mkdir()
    return root


def make_module_skill(root, sid, **kw):
    d = root / sid
    d.mkdir()
    (d / "skill.json").write_text(json.dumps(manifest(sid, **kw)))
    (d / "skill.py").write_text(MODULE_SKILL)
    return str(d)


def make_process_skill(root, sid):
    d = root / sid
    d.mkdir()
    (d / "skill.json").write_text(json.dumps(manifest(sid, mode="process",
                                                      examples=("run the process",))))
    exe = d / "skill"
    exe.write_text(PROCESS_SKILL.format(py=sys.executable))
    exe.chmod(exe.stat().st_mode | stat.S_IEXEC)
    return str(d)


def new_manager(root, tmp_path, **kw):
    cfg = SkillManagerConfig(skills_dir=str(root), config_store=str(tmp_path / "cfg"), **kw)
    return SkillManager(cfg, DefaultSkillLoader(skills_root=str(root)))


def run(coro):
    return asyncio.run(coro)


def test_manifest_roundtrip_field_names():
    m = SkillManifest.from_dict(manifest("x", priority=3))
    s = json.loads(gojson.dumps(m.to_go()))
    assert s["intent_patterns"][0]["min_confidence"] == 0.5
    assert s["min_loqa_version"] == "0.1" and s["sandbox_mode"] == "none"
    assert "homepage" not in s and "config_schema" not in s
    assert m.max_priority() == 3


def test_lights_skill_behaviour():
    s = LightsSkill()
    run(s.initialize(None))
    assert s.can_handle(VoiceIntent(transcript="Turn on the kitchen lights"))
    assert not s.can_handle(VoiceIntent(transcript="what's the weather"))
    assert parse_lighting("turn off the bedroom lights") == ("off", "bedroom")
    assert parse_lighting("dim the living room lamp") == ("dim", "living_room")
    assert parse_lighting("lights") == ("toggle", "main")
    r = run(s.handle_intent(VoiceIntent(transcript="switch on the lights everywhere")))
    assert r.success and r.message == "Turned on the lights in the all"
    assert r.speech_text == "Turned on the lights in the all in the all"
    assert r.actions[0].target == "lights.all" and r.actions[0].parameters == {"action": "on"}
    assert s.get_status().usage_count == 1
    m = s.get_manifest()
    assert m.id == "builtin.lights" and len(m.intent_patterns) == 4
    assert s.get_config_schema().properties["default_brightness"].default == 80


def test_builtin_executor_idempotent():
    ex = default_builtin_executor()
    m = SkillManifest(id="builtin.lights")
    a, b = ex.load_skill(m), ex.load_skill(m)
    assert a is b and ex.list_loaded_skills() == ["builtin.lights"]
    ex.unload_skill("builtin.lights")
    assert ex.list_loaded_skills() == []
    with pytest.raises(KeyError):
        BuiltinExecutor().load_skill(m)


def test_validate_skill_path(tmp_path):
    root = tmp_path / "skills"
    validate_skill_path(str(root / "a"), str(root))
    with pytest.raises(ValueError):
        validate_skill_path(str(tmp_path / "other"), str(root))
    assert contains_words("please turn on the lights", "turn on lights")
    assert not contains_words("turn off", "turn on")


def test_manager_load_route_unload(skills_root, tmp_path):
    async def go():
        mgr = new_manager(skills_root, tmp_path)
        path = make_module_skill(skills_root, "echo")
        await mgr.load_skill(path)
        with pytest.raises(SkillAlreadyLoaded):
            await mgr.load_skill(path)
        r = await mgr.handle_intent(VoiceIntent(transcript="echo hi"))
        assert r.message == "echo:echo hi"
        info = mgr.get_skill("echo")
        assert info.status.usage_count == 1 and info.config.enabled
        with pytest.raises(NoSkillCanHandle):
            await mgr.handle_intent(VoiceIntent(transcript="nothing"))
        await mgr.disable_skill("echo")
        assert mgr.get_skill("echo").status.state == SkillState.DISABLED
        with pytest.raises(NoSkillCanHandle):
            await mgr.handle_intent(VoiceIntent(transcript="echo hi"))
        saved = json.loads((tmp_path / "cfg" / "echo.json").read_text())
        assert saved["enabled"] is False and saved["timeout"] == 30 * 10**9
        await mgr.enable_skill("echo")
        # failing handler -> error recorded, "all candidates failed"
        with pytest.raises(Exception, match="all candidate skills failed"):
            await mgr.handle_intent(VoiceIntent(transcript="echo fail"))
        assert mgr.get_skill("echo").error_count == 1
        await mgr.unload_skill("echo")
        with pytest.raises(SkillNotFound):
            mgr.get_skill("echo")
        # persisted config is picked up on reload
        await mgr.load_skill(path)
        assert mgr.get_skill("echo").config.enabled is True
    run(go())


def test_manager_guards(skills_root, tmp_path):
    async def go():
        mgr = new_manager(skills_root, tmp_path, max_skills=1)
        with pytest.raises(Exception, match="path traversal"):
            await mgr.load_skill(str(skills_root / ".." / "x"))
        bad = skills_root / "bad"
        bad.mkdir()
        (bad / "skill.json").write_text(json.dumps({"id": "bad", "name": ""}))
        with pytest.raises(InvalidManifest):
            await mgr.load_skill(str(bad))
        wasm = skills_root / "w"
        wasm.mkdir()
        (wasm / "skill.json").write_text(json.dumps(manifest("w", mode="wasm")))
        with pytest.raises(Exception, match="sandbox mode wasm not supported"):
            await mgr.load_skill(str(wasm))
        await mgr.load_skill(make_module_skill(skills_root, "one"))
        with pytest.raises(Exception, match="maximum number of skills"):
            await mgr.load_skill(make_module_skill(skills_root, "two"))
        with pytest.raises(Exception):
            mgr.safe_config_path("../etc")
    run(go())


def test_manager_priority_order(skills_root, tmp_path):
    async def go():
        mgr = new_manager(skills_root, tmp_path)
        await mgr.load_skill(make_module_skill(skills_root, "low", priority=1))
        await mgr.load_skill(make_module_skill(skills_root, "high", priority=9))
        c = mgr.candidates(VoiceIntent(transcript="echo"))
        assert [x.info.manifest.id for x in c] == ["high", "low"]
        assert [i.manifest.name for i in mgr.list_skills()] == ["High", "Low"]
        assert mgr.get_skill("low").manifest.trust_level == "unknown"
    run(go())


def test_process_skill(skills_root, tmp_path):
    async def go():
        mgr = new_manager(skills_root, tmp_path)
        await mgr.load_skill(make_process_skill(skills_root, "proc"))
        r = await mgr.handle_intent(VoiceIntent(transcript="please run the process now"))
        assert r.message == "proc:please run the process now" and r.speech_text == "done"
        await mgr.stop()
        assert mgr.skills == {}
    run(go())


SLOW_PROCESS_SKILL = textwrap.dedent('''\
    #!{py}
    import json, sys, time
    for line in sys.stdin:
        req = json.loads(line)
        t = req["params"]["transcript"] if req["method"] == "handle_intent" else ""
        if "slow" in t:
            time.sleep(1.0)
        res = {{"success": True, "message": "proc:" + t}}
        sys.stdout.write(json.dumps({{"id": req["id"], "result": res}}) + "\\n")
        sys.stdout.flush()
''')


def test_process_skill_recovers_after_timeout(skills_root, tmp_path):
    """A timed-out call must not leave its late reply for the next call
    (every later call would read the previous reply)."""
    from loqa_hub_amd.skills.loader import ProcessSkill

    d = skills_root / "slow"
    d.mkdir()
    (d / "skill.json").write_text(json.dumps(manifest("slow", mode="process")))
    exe = d / "skill"
    exe.write_text(SLOW_PROCESS_SKILL.format(py=sys.executable))
    exe.chmod(exe.stat().st_mode | stat.S_IEXEC)

    async def go():
        sk = ProcessSkill(SkillManifest.from_dict(manifest("slow", mode="process")), str(exe),
                          str(d), request_timeout=0.3)
        r = await sk.handle_intent(VoiceIntent(transcript="fast one"))
        assert r.message == "proc:fast one"
        first = sk._proc
        with pytest.raises(asyncio.TimeoutError):
            await sk.handle_intent(VoiceIntent(transcript="slow one"))
        assert sk._proc is None and first.returncode is not None   # killed and reaped
        for k in range(3):   # respawned; replies line up with their requests again
            r = await sk.handle_intent(VoiceIntent(transcript=f"fast {k}"))
            assert r.message == f"proc:fast {k}"
        await sk.close()
    run(go())


def test_auto_load_all(skills_root, tmp_path):
    async def go():
        make_module_skill(skills_root, "a1")
        make_module_skill(skills_root, "a2")
        (skills_root / "empty").mkdir()
        mgr = new_manager(skills_root, tmp_path)
        await mgr.start()
        assert sorted(mgr.skills) == ["a1", "a2"]
        await mgr.stop()
    run(go())


def test_skills_api(skills_root, tmp_path):
    async def go():
        mgr = new_manager(skills_root, tmp_path)
        app = web.Application()
        app.add_routes(SkillsHandler(mgr).routes())
        async with TestClient(TestServer(app)) as c:
            r = await c.get("/api/skills")
            assert r.status == 200 and (await r.json()) == {"count": 0, "skills": []}
            path = make_module_skill(skills_root, "echo")
            r = await c.post("/api/skills", data=json.dumps({"skill_path": path}))
            assert r.status == 201 and (await r.json())["path"] == path
            r = await c.post("/api/skills", data=json.dumps({"skill_path": path}))
            assert r.status == 409 and (await r.json()) == {"error": True,
                                                            "message": "skill already loaded"}
            r = await c.post("/api/skills", data="nope")
            assert r.status == 400
            r = await c.post("/api/skills", data="{}")
            assert (await r.json())["message"] == "skill_path is required"
            r = await c.get("/api/skills/echo")
            body = await r.json()
            assert r.status == 200 and body["manifest"]["id"] == "echo"
            assert body["config"]["timeout"] == 30 * 10**9 and body["plugin_path"] == path
            assert (await c.get("/api/skills/missing")).status == 404
            assert (await c.get("/api/skills/bad.id")).status == 400
            r = await c.post("/api/skills/echo/disable")
            assert (await r.json()) == {"message": "skill disabled successfully", "skill": "echo"}
            assert (await c.post("/api/skills/echo/explode")).status == 400
            assert (await c.get("/api/skills/echo/enable")).status == 405
            r = await c.post("/api/skills/echo/reload")
            assert r.status == 200
            r = await c.put("/api/skills/echo", data=json.dumps({"config": {"k": 1}}))
            assert r.status == 200 and mgr.get_skill("echo").config.config == {"k": 1}
            r = await c.delete("/api/skills/echo")
            assert r.status == 200
            assert (await c.delete("/api/skills/echo")).status == 404
            assert (await c.patch("/api/skills")).status == 405
    run(go())
