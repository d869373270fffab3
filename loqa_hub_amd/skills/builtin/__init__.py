"""Builtin skills shipped with the hub."""
from .lights import LightsSkill

__all__ = ["LightsSkill"]
