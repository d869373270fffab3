"""Command data model and LLM-response parsing.

Behavioural spec: ``internal/llm/command_parser.go`` -
``Command``/``MultiCommand`` (:45-58), ``parseResponse`` (:269-303),
``detectCompoundUtterance`` (:306-336), ``parseMultiCommandResponse`` (:413-473),
``createCombinedCommand`` (:476-516). Parsing keeps the reference's
"first ``{`` to last ``}``" extraction and default-filling so output from an
unconstrained backend (e.g. a real Ollama in config 1) is handled identically;
the GPU backend's grammar-constrained output always passes it.
"""
from __future__ import annotations

import json
import re
from dataclasses import dataclass, field

from .prompts import DEFAULT_UNCLEAR_RESPONSE


@dataclass
class Command:
    intent: str = "unknown"
    entities: dict[str, str] = field(default_factory=dict)
    confidence: float = 0.0
    response: str = ""

    def to_dict(self) -> dict:
        return {"intent": self.intent, "entities": dict(self.entities),
                "confidence": self.confidence, "response": self.response}


@dataclass
class MultiCommand:
    commands: list[Command] = field(default_factory=list)
    is_multi: bool = False
    original_text: str = ""
    combined_response: str = ""

    def to_dict(self) -> dict:
        return {"commands": [c.to_dict() for c in self.commands], "is_multi": self.is_multi,
                "original_text": self.original_text, "combined_response": self.combined_response}


class ParseError(ValueError):
    pass


CONJUNCTION_PATTERNS = [
    " and ", " then ", " after that ", " next ", " also ",
    ", and ", ", then ", ", after that ", ", next ", ", also ",
    " and then ", " then also ", " and also ",
]
EXCLUSION_PATTERNS = [
    "rock and roll", "rhythm and blues", "black and white", "salt and pepper",
    "peanut butter and jelly", "research and development", "arts and crafts",
]


def detect_compound_utterance(text: str) -> bool:
    low = text.lower()
    if any(e in low for e in EXCLUSION_PATTERNS):
        return False
    return any(p in low for p in CONJUNCTION_PATTERNS)


_SPLIT_RE = re.compile(
    "|".join(re.escape(p) for p in sorted(CONJUNCTION_PATTERNS, key=len, reverse=True)),
    re.IGNORECASE)


def split_compound_utterance(text: str) -> list[str]:
    """Split a compound utterance into command clauses on the same conjunction
    set the detector uses (longest pattern first). Used to fix the number of
    command objects in the constrained decode; a single clause for
    non-compound text."""
    if not detect_compound_utterance(text):
        return [text.strip()] if text.strip() else []
    parts = [p.strip(" ,.") for p in _SPLIT_RE.split(" " + text + " ")]
    return [p for p in parts if p]


def _extract_json(response: str, what: str) -> dict:
    response = response.strip()
    start, end = response.find("{"), response.rfind("}")
    if start == -1 or end == -1 or start >= end:
        raise ParseError(f"no valid JSON found in {what}")
    try:
        obj = json.loads(response[start:end + 1])
    except json.JSONDecodeError as e:
        raise ParseError(f"error unmarshaling {what} JSON: {e}") from e
    if not isinstance(obj, dict):
        raise ParseError(f"{what} JSON is not an object")
    return obj


def _command_from(obj: dict) -> Command:
    ents = obj.get("entities")
    if not isinstance(ents, dict):
        ents = {}
    ents = {str(k): ("" if v is None else str(v)) for k, v in ents.items()}
    try:
        conf = float(obj.get("confidence", 0.0) or 0.0)
    except (TypeError, ValueError):
        conf = 0.0
    cmd = Command(intent=str(obj.get("intent") or ""), entities=ents, confidence=conf,
                  response=str(obj.get("response") or ""))
    if not cmd.intent:
        cmd.intent = "unknown"
    if cmd.confidence < 0 or cmd.confidence > 1:
        cmd.confidence = 0.5
    if not cmd.response:
        cmd.response = DEFAULT_UNCLEAR_RESPONSE
    return cmd


def parse_response(response: str) -> Command:
    return _command_from(_extract_json(response, "response"))


def parse_multi_command_response(response: str, original_text: str) -> MultiCommand:
    obj = _extract_json(response, "multi-command response")
    raw = obj.get("commands") or []
    if not isinstance(raw, list):
        raise ParseError("commands is not a list")
    cmds = [_command_from(c if isinstance(c, dict) else {}) for c in raw]
    combined = str(obj.get("combined_response") or "")
    if not combined:
        if len(cmds) > 1:
            combined = "I'll handle those commands for you."
        elif len(cmds) == 1:
            combined = cmds[0].response
        else:
            combined = DEFAULT_UNCLEAR_RESPONSE
    return MultiCommand(commands=cmds, is_multi=bool(obj.get("is_multi")) and len(cmds) > 1,
                        original_text=original_text, combined_response=combined)


def create_combined_command(mc: MultiCommand) -> Command:
    if not mc.commands:
        return Command("unknown", {}, 0.0, DEFAULT_UNCLEAR_RESPONSE)
    if len(mc.commands) == 1:
        return mc.commands[0]
    ents: dict[str, str] = {}
    total = 0.0
    for c in mc.commands:
        for k, v in c.entities.items():
            ents[k] = ents[k] + ", " + v if k in ents else v
        total += c.confidence
    return Command("multi_" + mc.commands[0].intent, ents, total / len(mc.commands),
                   mc.combined_response)
