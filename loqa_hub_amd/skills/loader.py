"""Skill loader (``internal/skills/loader.go``).

Sandbox modes (loader.go:79-110):

* ``none``    - in-process plugin. The reference ``plugin.Open``s ``skill.so`` /
                ``<id>.so`` and looks up ``NewSkill`` (:121-155); the Python
                equivalent imports ``skill.py`` / ``<id>.py`` from the skill
                directory and calls its ``new_skill()`` factory.
* ``process`` - out-of-process plugin: executable ``skill``, ``skill.exe``,
                ``<id>`` or ``<id>.exe`` (:158-188). The reference's
                ``ProcessSkill`` is a stub that answers "Hello from <name>" and
                whose ``containsWords`` is always true (:191-272). Here it is a
                real child process speaking JSON lines over stdin/stdout::

                    -> {"id": 1, "method": "handle_intent", "params": {...VoiceIntent}}
                    <- {"id": 1, "result": {...SkillResponse}}   |  {"id": 1, "error": "..."}

                methods: ``initialize`` (params = SkillConfig), ``handle_intent``,
                ``update_config``, ``health_check``, ``teardown``. ``can_handle``
                matches the manifest's intent-pattern examples word-by-word
                (every example word present in the transcript).
* ``wasm`` / ``docker`` - not implemented (same as the reference).

Skill directories must live under ``skills_root`` (default ``./skills``,
:35-56).
"""
from __future__ import annotations

import asyncio
import importlib.util
import itertools
import json
import logging
import os
import re
import sys

from ..utils import gojson
from ..utils.security import sanitize_log_input
from .interfaces import (SandboxMode, SkillConfig, SkillManifest, SkillPlugin, SkillResponse,
                         SkillState, SkillStatus, VoiceIntent)

log = logging.getLogger("loqa.skills.loader")

SKILLS_ROOT_DIR = "./skills"


def validate_skill_path(skill_path: str, root: str = SKILLS_ROOT_DIR) -> None:
    p = os.path.abspath(skill_path)
    r = os.path.abspath(root)
    if not (p.startswith(r + os.sep) or p == r):
        raise ValueError(f"skill path {skill_path!r} is outside the allowed skills directory {root!r}")


def _read_manifest(skill_path: str) -> SkillManifest:
    with open(os.path.normpath(os.path.join(skill_path, "skill.json")), "rb") as f:
        return SkillManifest.from_dict(json.loads(f.read()))


_WORD = re.compile(r"[a-z0-9']+")


def contains_words(text: str, pattern: str) -> bool:
    words = set(_WORD.findall(text.lower()))
    pw = _WORD.findall(pattern.lower())
    return bool(pw) and all(w in words for w in pw)


class DefaultSkillLoader:
    def __init__(self, skills_root: str = SKILLS_ROOT_DIR):
        self.skills_root = skills_root
        self._modes = [SandboxMode.NONE, SandboxMode.PROCESS]

    def supported_modes(self) -> list[str]:
        return list(self._modes)

    async def load_skill(self, skill_path: str) -> SkillPlugin:
        try:
            validate_skill_path(skill_path, self.skills_root)
        except ValueError as e:
            raise ValueError(f"invalid skill path: {e}") from e
        m = _read_manifest(skill_path)
        if m.sandbox_mode == SandboxMode.NONE:
            return self._load_module(skill_path, m)
        if m.sandbox_mode == SandboxMode.PROCESS:
            return self._load_process(skill_path, m)
        if m.sandbox_mode == SandboxMode.WASM:
            raise NotImplementedError("wasm sandbox mode not implemented")
        if m.sandbox_mode == SandboxMode.DOCKER:
            raise NotImplementedError("docker sandbox mode not implemented")
        raise ValueError(f"unsupported sandbox mode: {m.sandbox_mode}")

    async def unload_skill(self, plugin: SkillPlugin) -> None:
        if isinstance(plugin, ProcessSkill):
            await plugin.close()

    def _load_module(self, skill_path: str, m: SkillManifest) -> SkillPlugin:
        path = os.path.join(skill_path, "skill.py")
        if not os.path.isfile(path):
            path = os.path.join(skill_path, m.id + ".py")
            if not os.path.isfile(path):
                raise FileNotFoundError(f"plugin file not found in {skill_path}")
        modname = f"loqa_skill_{m.id.replace('-', '_')}_{abs(hash(os.path.abspath(path)))}"
        spec = importlib.util.spec_from_file_location(modname, path)
        if spec is None or spec.loader is None:
            raise ImportError(f"failed to open plugin {path}")
        mod = importlib.util.module_from_spec(spec)
        sys.modules[modname] = mod
        try:
            spec.loader.exec_module(mod)
        except Exception:
            sys.modules.pop(modname, None)
            raise
        factory = getattr(mod, "new_skill", None)
        if factory is None:
            raise ImportError("new_skill symbol not found in plugin")
        skill = factory()
        if not isinstance(skill, SkillPlugin):
            raise TypeError("new_skill has incorrect signature")
        log.info("Loaded module plugin skill=%s path=%s", sanitize_log_input(m.id), path)
        return skill

    def _load_process(self, skill_path: str, m: SkillManifest) -> SkillPlugin:
        for cand in ("skill", "skill.exe", m.id, m.id + ".exe"):
            p = os.path.join(skill_path, cand)
            if os.path.isfile(p):
                log.info("Loaded process plugin skill=%s path=%s", sanitize_log_input(m.id), p)
                return ProcessSkill(m, p, skill_path)
        raise FileNotFoundError(f"skill executable not found in {skill_path}")


class ProcessSkill(SkillPlugin):
    def __init__(self, manifest: SkillManifest, exec_path: str, skill_path: str,
                 request_timeout: float = 30.0):
        self.manifest, self.exec_path, self.skill_path = manifest, exec_path, skill_path
        self.config: SkillConfig | None = None
        self.status = SkillStatus(SkillState.LOADING, False)
        self.request_timeout = request_timeout
        self._proc: asyncio.subprocess.Process | None = None
        self._ids = itertools.count(1)
        self._io = asyncio.Lock()

    async def _spawn(self) -> None:
        argv = [self.exec_path]
        if self.exec_path.endswith(".py"):
            argv = [sys.executable, self.exec_path]
        self._proc = await asyncio.create_subprocess_exec(
            *argv, cwd=self.skill_path, stdin=asyncio.subprocess.PIPE,
            stdout=asyncio.subprocess.PIPE, stderr=asyncio.subprocess.DEVNULL)

    async def call(self, method: str, params) -> dict | None:
        """One request/reply. A timeout, a garbled or out-of-order reply, or a
        cancelled call leaves the child's stdout in an unknown state (a late
        reply would be read by the NEXT call), so the child is killed and
        reaped and the next call respawns it."""
        async with self._io:
            if self._proc is None or self._proc.returncode is not None:
                await self._spawn()
            rid = next(self._ids)
            msg = '{"id":%d,"method":%s,"params":%s}\n' % (rid, json.dumps(method),
                                                           gojson.dumps(params))
            try:
                self._proc.stdin.write(msg.encode())
                await self._proc.stdin.drain()
                line = await asyncio.wait_for(self._proc.stdout.readline(), self.request_timeout)
                if not line:
                    raise RuntimeError(f"skill process {self.manifest.id} exited")
                try:
                    resp = json.loads(line)
                except ValueError as e:
                    raise RuntimeError(f"skill process protocol error: {e}") from e
                if not isinstance(resp, dict) or resp.get("id") != rid:
                    raise RuntimeError("skill process protocol error: id mismatch")
            except BaseException:
                await self._kill()
                raise
            if resp.get("error"):
                raise RuntimeError(str(resp["error"]))
            return resp.get("result")

    async def _kill(self) -> None:
        p, self._proc = self._proc, None
        if p is not None and p.returncode is None:
            try:
                p.kill()
            except ProcessLookupError:
                pass
            await p.wait()

    async def initialize(self, config: SkillConfig) -> None:
        self.config = config
        await self.call("initialize", config.to_go())
        self.status = SkillStatus(SkillState.READY, True)

    async def teardown(self) -> None:
        try:
            if self._proc is not None and self._proc.returncode is None:
                await self.call("teardown", None)
        finally:
            self.status = SkillStatus(SkillState.SHUTDOWN, False)
            await self.close()

    async def close(self) -> None:
        p, self._proc = self._proc, None
        if p is not None and p.returncode is None:
            try:
                p.stdin.close()
                await asyncio.wait_for(p.wait(), 2.0)
            except (asyncio.TimeoutError, ProcessLookupError, BrokenPipeError):
                p.kill()
                await p.wait()

    def can_handle(self, intent: VoiceIntent) -> bool:
        return any(contains_words(intent.transcript, ex)
                   for p in self.manifest.intent_patterns for ex in p.examples)

    async def handle_intent(self, intent: VoiceIntent) -> SkillResponse:
        res = await self.call("handle_intent", intent.to_go())
        return SkillResponse.from_dict(res or {})

    def get_manifest(self) -> SkillManifest:
        return self.manifest

    def get_status(self) -> SkillStatus:
        return self.status

    def get_config(self) -> SkillConfig | None:
        return self.config

    async def update_config(self, config: SkillConfig) -> None:
        self.config = config
        await self.call("update_config", config.to_go())

    async def health_check(self) -> None:
        await self.call("health_check", None)
