"""``SkillManagerInterface`` (``async_execution.go:52-55``) over the skill manager.

``find_skill_for_intent`` routes with the manager's ordered candidate list;
``execute_skill`` runs the plugin with the skill's configured timeout and
records usage. ``NullSkillManager`` is the reference's ``SkillManagerAdapter``
(``audio_service.go:294-342``) used when no skills are loaded.
"""
from __future__ import annotations

import asyncio
from datetime import datetime, timezone

from ..skills.interfaces import SkillPlugin, SkillResponse, VoiceIntent
from ..skills.manager import NoSkillCanHandle, SkillManager


class SkillManagerAdapter:
    def __init__(self, manager: SkillManager):
        self.manager = manager

    def find_skill_for_intent(self, intent: VoiceIntent) -> SkillPlugin:
        cands = self.manager.candidates(intent)
        if not cands:
            raise NoSkillCanHandle()
        return cands[0].plugin

    async def execute_skill(self, skill: SkillPlugin, intent: VoiceIntent) -> SkillResponse:
        info = next((ls.info for ls in self.manager.skills.values() if ls.plugin is skill), None)
        timeout = (info.config.timeout_s if info is not None else 0) or 30.0
        resp = await asyncio.wait_for(skill.handle_intent(intent), timeout)
        if info is not None:
            now = datetime.now(timezone.utc)
            info.last_used = now
            info.status.last_used = now
            info.status.usage_count += 1
        return resp


class NullSkillManager:
    def find_skill_for_intent(self, intent: VoiceIntent) -> SkillPlugin:
        raise LookupError("no skills available")

    async def execute_skill(self, skill, intent) -> SkillResponse:
        raise RuntimeError("skill execution not available")
