"""Skill lifecycle manager (``internal/skills/manager.go``).

Behaviour kept from the reference:
* errors: not found / already loaded / invalid manifest / no skill can handle
  (manager.go:38-46);
* limits: ``max_skills`` 50, ``load_timeout`` 30 s defaults (:112-125);
* ``load_skill`` (:162-252): path guard (no ``..`` / ``\\``), manifest load and
  validation (id/name/version required, id must pass ``validate_skill_id``),
  duplicate and capacity checks, sandbox-mode allow-list with default trust
  (:500-519), loader call under the load timeout, per-skill JSON config from the
  config store or defaults (enabled, 30 s timeout, 3 retries), ``initialize``
  with loader unload on failure;
* ``handle_intent`` (:290-346): candidates are ready + healthy + enabled +
  ``can_handle``; each runs under its config timeout, failures bump
  ``error_count`` / ``last_error`` and fall through to the next candidate;
* enable/disable persist the config to ``<config_store>/<id>.json`` through a
  path-traversal guard (:49-76, :522-562);
* ``load_all_skills`` scans ``skills_dir/*/skill.json`` one level deep (:438-461).

Deliberate fix: the reference's candidate "priority sort" is a no-op
(``return true``, :318-321); here candidates are ordered by the highest enabled
intent-pattern priority, then trust level (system > verified > community >
unknown), then skill id, so routing is deterministic.
"""
from __future__ import annotations

import asyncio
import json
import logging
import os
from dataclasses import dataclass, field, replace
from datetime import datetime, timezone

from ..utils.security import InvalidSkillID, sanitize_log_input, validate_skill_id
from .interfaces import (NS, TRUST_RANK, SandboxMode, SkillConfig, SkillInfo, SkillManifest,
                         SkillPlugin, SkillResponse, SkillState, SkillStatus, TrustLevel,
                         VoiceIntent)

log = logging.getLogger("loqa.skills")


class SkillError(Exception):
    pass


class SkillNotFound(SkillError):
    def __init__(self):
        super().__init__("skill not found")


class SkillAlreadyLoaded(SkillError):
    def __init__(self):
        super().__init__("skill already loaded")


class InvalidManifest(SkillError):
    def __init__(self, msg: str = "invalid skill manifest"):
        super().__init__(msg)


class PermissionDenied(SkillError):
    def __init__(self):
        super().__init__("permission denied")


class SkillInitFailed(SkillError):
    pass


class NoSkillCanHandle(SkillError):
    def __init__(self):
        super().__init__("no skill can handle this intent")


@dataclass
class SkillManagerConfig:
    skills_dir: str = "./skills"
    auto_load: bool = True
    max_skills: int = 50
    load_timeout_s: float = 30.0
    default_trust: str = TrustLevel.UNKNOWN
    allowed_modes: list[str] = field(default_factory=lambda: [SandboxMode.NONE,
                                                              SandboxMode.PROCESS])
    config_store: str = ""


class SkillLoaderProtocol:
    async def load_skill(self, skill_path: str) -> SkillPlugin: ...

    async def unload_skill(self, plugin: SkillPlugin) -> None: ...

    def supported_modes(self) -> list[str]: ...


@dataclass
class LoadedSkill:
    plugin: SkillPlugin
    info: SkillInfo


def default_skill_config(m: SkillManifest) -> SkillConfig:
    return SkillConfig(skill_id=m.id, name=m.name, version=m.version, config={},
                       permissions=list(m.permissions), enabled=True, timeout_ns=30 * NS,
                       max_retries=3)


def _priority_key(ls: LoadedSkill):
    m = ls.info.manifest
    return (-m.max_priority(), -TRUST_RANK.get(m.trust_level, 0), m.id)


class SkillManager:
    def __init__(self, config: SkillManagerConfig, loader: SkillLoaderProtocol):
        if config.max_skills <= 0:
            config.max_skills = 50
        if config.load_timeout_s <= 0:
            config.load_timeout_s = 30.0
        self.config = config
        self.loader = loader
        self.skills: dict[str, LoadedSkill] = {}
        self._lock = asyncio.Lock()

    # -- lifecycle --------------------------------------------------------------------------------
    async def start(self) -> None:
        log.info("Starting skill manager skills_dir=%s", sanitize_log_input(self.config.skills_dir))
        if self.config.auto_load:
            try:
                await self.load_all_skills()
            except OSError as e:
                log.warning("Failed to load some skills during startup: %s", e)

    async def stop(self) -> None:
        async with self._lock:
            errors = []
            for sid in list(self.skills):
                try:
                    await self._unload_unlocked(sid)
                except Exception as e:  # noqa: BLE001
                    errors.append(f"failed to unload skill {sid}: {e}")
            if errors:
                raise SkillError(f"errors during shutdown: {errors}")

    # -- load / unload ----------------------------------------------------------------------------
    async def load_skill(self, skill_path: str) -> None:
        async with self._lock:
            await self._load_unlocked(skill_path)

    async def _load_unlocked(self, skill_path: str) -> None:
        if not skill_path:
            raise SkillError("skill path cannot be empty")
        if ".." in skill_path or "\\" in skill_path:
            raise SkillError("invalid skill path: path traversal detected")
        try:
            manifest = self.load_manifest(skill_path)
        except InvalidManifest:
            raise
        except Exception as e:
            raise SkillError(f"failed to load manifest: {e}") from e
        if manifest.id in self.skills:
            raise SkillAlreadyLoaded()
        if len(self.skills) >= self.config.max_skills:
            raise SkillError(f"maximum number of skills reached: {self.config.max_skills}")
        self.validate_skill(manifest)
        try:
            plugin = await asyncio.wait_for(self.loader.load_skill(skill_path),
                                            self.config.load_timeout_s)
        except Exception as e:
            raise SkillError(f"failed to load skill plugin: {e}") from e
        try:
            config = self.load_skill_config(manifest.id)
        except Exception as e:  # noqa: BLE001 - missing/invalid config -> defaults
            log.debug("using default config for %s: %s", sanitize_log_input(manifest.id), e)
            config = default_skill_config(manifest)
        try:
            await asyncio.wait_for(plugin.initialize(config), self.config.load_timeout_s)
        except Exception as e:
            try:
                await self.loader.unload_skill(plugin)
            except Exception as ue:  # noqa: BLE001
                log.warning("Failed to unload skill after initialization failure: %s", ue)
            raise SkillInitFailed(f"skill initialization failed: {e}") from e
        info = SkillInfo(manifest=manifest, config=config,
                         status=SkillStatus(state=SkillState.READY, healthy=True),
                         loaded_at=datetime.now(timezone.utc), plugin_path=skill_path)
        self.skills[manifest.id] = LoadedSkill(plugin, info)
        log.info("Skill loaded successfully skill_id=%s name=%s version=%s",
                 sanitize_log_input(manifest.id), sanitize_log_input(manifest.name),
                 sanitize_log_input(manifest.version))

    async def register_plugin(self, plugin: SkillPlugin, *, plugin_path: str = "builtin") -> None:
        """Load an in-process (builtin) plugin without a manifest file; used for
        the builtin executor's skills, which the reference also constructs directly."""
        m = plugin.get_manifest()
        async with self._lock:
            if m.id in self.skills:
                raise SkillAlreadyLoaded()
            if len(self.skills) >= self.config.max_skills:
                raise SkillError(f"maximum number of skills reached: {self.config.max_skills}")
            if not m.trust_level:
                m.trust_level = self.config.default_trust
            try:
                config = self.load_skill_config(m.id)
            except Exception:  # noqa: BLE001
                config = default_skill_config(m)
            await plugin.initialize(config)
            self.skills[m.id] = LoadedSkill(plugin, SkillInfo(
                manifest=m, config=config, status=SkillStatus(SkillState.READY, True),
                loaded_at=datetime.now(timezone.utc), plugin_path=plugin_path))

    async def unload_skill(self, skill_id: str) -> None:
        async with self._lock:
            await self._unload_unlocked(skill_id)

    async def _unload_unlocked(self, skill_id: str) -> None:
        ls = self.skills.get(skill_id)
        if ls is None:
            raise SkillNotFound()
        ls.info.status.state = SkillState.SHUTDOWN
        try:
            await ls.plugin.teardown()
        except Exception as e:  # noqa: BLE001
            log.warning("Skill teardown failed skill=%s: %s", sanitize_log_input(skill_id), e)
        try:
            await self.loader.unload_skill(ls.plugin)
        except Exception as e:  # noqa: BLE001
            log.warning("Failed to unload skill from loader skill=%s: %s",
                        sanitize_log_input(skill_id), e)
        del self.skills[skill_id]

    async def reload_skill(self, skill_id: str) -> None:
        async with self._lock:
            ls = self.skills.get(skill_id)
            if ls is None:
                raise SkillNotFound()
            path = ls.info.plugin_path
            await self._unload_unlocked(skill_id)
            await self._load_unlocked(path)

    # -- routing ----------------------------------------------------------------------------------
    def candidates(self, intent: VoiceIntent) -> list[LoadedSkill]:
        out = []
        for ls in self.skills.values():
            st, cfg = ls.info.status, ls.info.config
            if st.state == SkillState.READY and st.healthy and cfg.enabled:
                try:
                    if ls.plugin.can_handle(intent):
                        out.append(ls)
                except Exception as e:  # noqa: BLE001
                    log.warning("can_handle raised in %s: %s", ls.info.manifest.id, e)
        out.sort(key=_priority_key)
        return out

    async def handle_intent(self, intent: VoiceIntent) -> SkillResponse:
        cands = self.candidates(intent)
        if not cands:
            raise NoSkillCanHandle()
        last: Exception | None = None
        for c in cands:
            timeout = c.info.config.timeout_s or 30.0
            try:
                resp = await asyncio.wait_for(c.plugin.handle_intent(intent), timeout)
            except Exception as e:  # noqa: BLE001
                last = e if not isinstance(e, asyncio.TimeoutError) else \
                    SkillError("context deadline exceeded")
                c.info.error_count += 1
                c.info.last_error = str(last)
                log.warning("Skill execution failed skill=%s error=%s",
                            sanitize_log_input(c.info.manifest.id), last)
                continue
            now = datetime.now(timezone.utc)
            c.info.last_used = now
            c.info.status.last_used = now
            c.info.status.usage_count += 1
            return resp
        raise SkillError(f"all candidate skills failed, last error: {last}")

    # -- queries ----------------------------------------------------------------------------------
    def get_skill(self, skill_id: str) -> SkillInfo:
        ls = self.skills.get(skill_id)
        if ls is None:
            raise SkillNotFound()
        return replace(ls.info)  # shallow copy; config object shared like the reference

    def list_skills(self) -> list[SkillInfo]:
        infos = [replace(ls.info) for ls in self.skills.values()]
        infos.sort(key=lambda i: i.manifest.name)
        return infos

    async def enable_skill(self, skill_id: str) -> None:
        await self._set_enabled(skill_id, True)

    async def disable_skill(self, skill_id: str) -> None:
        await self._set_enabled(skill_id, False)

    async def _set_enabled(self, skill_id: str, enabled: bool) -> None:
        ls = self.skills.get(skill_id)
        if ls is None:
            raise SkillNotFound()
        ls.info.config.enabled = enabled
        ls.info.status.state = SkillState.READY if enabled else SkillState.DISABLED
        try:
            await ls.plugin.update_config(ls.info.config)
        except Exception as e:
            raise SkillError(f"failed to update skill config: {e}") from e
        try:
            self.save_skill_config(skill_id, ls.info.config)
        except Exception as e:  # noqa: BLE001
            log.warning("Failed to save skill config skill=%s: %s", sanitize_log_input(skill_id), e)

    async def update_skill_config(self, skill_id: str, values: dict) -> None:
        ls = self.skills.get(skill_id)
        if ls is None:
            raise SkillNotFound()
        ls.info.config.config = dict(values)
        await ls.plugin.update_config(ls.info.config)
        try:
            self.save_skill_config(skill_id, ls.info.config)
        except Exception as e:  # noqa: BLE001
            log.warning("Failed to save skill config skill=%s: %s", sanitize_log_input(skill_id), e)

    # -- files ------------------------------------------------------------------------------------
    async def load_all_skills(self) -> None:
        root = self.config.skills_dir
        if not root or not os.path.isdir(root):
            return
        for name in sorted(os.listdir(root)):
            path = os.path.join(root, name)
            if os.path.isdir(path) and os.path.isfile(os.path.join(path, "skill.json")):
                try:
                    await self.load_skill(path)
                except Exception as e:  # noqa: BLE001
                    log.warning("Failed to load skill path=%s: %s", sanitize_log_input(path), e)

    @staticmethod
    def load_manifest(skill_path: str) -> SkillManifest:
        if not skill_path:
            raise SkillError("empty skill path")
        if ".." in skill_path:
            raise SkillError("invalid skill path: path traversal detected")
        with open(os.path.normpath(os.path.join(skill_path, "skill.json")), "rb") as f:
            data = f.read()
        try:
            m = SkillManifest.from_dict(json.loads(data))
        except ValueError as e:
            raise SkillError(f"failed to parse manifest: {e}") from e
        if not (m.id and m.name and m.version):
            raise InvalidManifest()
        try:
            validate_skill_id(m.id)
        except InvalidSkillID as e:
            raise InvalidManifest(f"invalid skill ID in manifest: {e}") from e
        return m

    def validate_skill(self, m: SkillManifest) -> None:
        if m.sandbox_mode not in self.config.allowed_modes:
            raise SkillError(f"skill validation failed: sandbox mode {m.sandbox_mode} not supported")
        if not m.trust_level:
            m.trust_level = self.config.default_trust

    def safe_config_path(self, skill_id: str) -> str:
        validate_skill_id(skill_id)
        safe_dir = os.path.abspath(self.config.config_store)
        p = os.path.abspath(os.path.join(safe_dir, skill_id + ".json"))
        if not p.startswith(safe_dir + os.sep):
            raise SkillError("invalid file path: path traversal detected")
        return p

    def load_skill_config(self, skill_id: str) -> SkillConfig:
        if not self.config.config_store:
            raise FileNotFoundError("no config store")
        with open(self.safe_config_path(skill_id), "rb") as f:
            return SkillConfig.from_dict(json.loads(f.read()))

    def save_skill_config(self, skill_id: str, config: SkillConfig) -> None:
        if not self.config.config_store:
            return
        os.makedirs(self.config.config_store, mode=0o750, exist_ok=True)
        path = self.safe_config_path(skill_id)
        from ..utils import gojson
        data = json.dumps(json.loads(gojson.dumps(config.to_go())), indent=2)
        fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o600)
        with os.fdopen(fd, "w") as f:
            f.write(data)
