"""Registry of in-process builtin skills (``internal/skills/builtin_executor.go``).

``register_skill(id, factory)`` records a factory; ``load_skill`` instantiates it
once and returns the same instance on later calls (idempotent, :58-82).
"""
from __future__ import annotations

import logging
import threading
from typing import Callable

from .interfaces import SkillConfig, SkillExecutor, SkillManifest, SkillPlugin

log = logging.getLogger("loqa.skills.builtin")

SkillFactory = Callable[[], SkillPlugin]


class BuiltinExecutor(SkillExecutor):
    def __init__(self):
        self._registry: dict[str, SkillFactory] = {}
        self._loaded: dict[str, SkillPlugin] = {}
        self._lock = threading.RLock()

    def register_skill(self, skill_id: str, factory: SkillFactory) -> None:
        with self._lock:
            self._registry[skill_id] = factory
        log.info("Registered built-in skill %s", skill_id)

    def load_skill(self, manifest: SkillManifest, config: SkillConfig | None = None) -> SkillPlugin:
        with self._lock:
            if manifest.id in self._loaded:
                return self._loaded[manifest.id]
            factory = self._registry.get(manifest.id)
            if factory is None:
                raise KeyError(f"built-in skill {manifest.id} not registered")
            skill = factory()
            self._loaded[manifest.id] = skill
            return skill

    def unload_skill(self, skill_id: str) -> None:
        with self._lock:
            self._loaded.pop(skill_id, None)

    def list_loaded_skills(self) -> list[str]:
        with self._lock:
            return list(self._loaded)


def default_builtin_executor() -> BuiltinExecutor:
    from .builtin.lights import LightsSkill
    ex = BuiltinExecutor()
    ex.register_skill("builtin.lights", LightsSkill)
    return ex
