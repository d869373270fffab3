"""Skill plugin system: contract, manager, loaders, builtins (``internal/skills``)."""
from .builtin_executor import BuiltinExecutor, default_builtin_executor
from .interfaces import (ConfigProperty, ConfigSchema, IntentPattern, Permission, PermissionType,
                         SandboxMode, SkillAction, SkillConfig, SkillExecutor, SkillInfo,
                         SkillManifest, SkillPlugin, SkillResponse, SkillState, SkillStatus,
                         TrustLevel, VoiceIntent)
from .loader import DefaultSkillLoader, ProcessSkill, validate_skill_path
from .manager import (InvalidManifest, NoSkillCanHandle, SkillAlreadyLoaded, SkillError,
                      SkillInitFailed, SkillManager, SkillManagerConfig, SkillNotFound)

__all__ = [n for n in dir() if not n.startswith("_")]
