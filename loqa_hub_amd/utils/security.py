"""Input hygiene (``internal/security/security.go``).

* ``sanitize_log_input`` strips ``\\n``/``\\r`` from user-controlled strings
  before they reach a log line (log-injection guard, :37-41).
* ``validate_skill_id`` allows only ``^[a-zA-Z0-9_-]+$`` and rejects path
  separators and ``..`` (path-traversal guard, :46-63).
"""
from __future__ import annotations

import re

_SKILL_ID = re.compile(r"^[a-zA-Z0-9_-]+$")


class InvalidSkillID(ValueError):
    def __init__(self, msg: str = "invalid skill ID"):
        super().__init__(msg)


def sanitize_log_input(s: str) -> str:
    return str(s).replace("\n", "").replace("\r", "")


def validate_skill_id(skill_id: str) -> None:
    if not skill_id:
        raise InvalidSkillID()
    if "/" in skill_id or "\\" in skill_id or ".." in skill_id:
        raise InvalidSkillID()
    if not _SKILL_ID.fullmatch(skill_id):
        raise InvalidSkillID()
