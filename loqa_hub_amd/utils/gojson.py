"""JSON encoding byte-compatible with Go's ``encoding/json.Marshal``.

The hub's NATS payloads and HTTP bodies must stay byte-identical to the
reference's so existing relays/skills/devices keep working:
compact separators, map keys sorted, HTML-significant characters escaped
(``<`` ``>`` ``&`` -> ``\\u003c`` ...), U+2028/2029 escaped, floats in Go's
shortest 'f'/'e' form (``1`` not ``1.0``), ``[]byte`` as base64.
"""
from __future__ import annotations

import base64
import json
import math


def go_float(f: float) -> str:
    if math.isnan(f) or math.isinf(f):
        raise ValueError("json: unsupported value: NaN/Inf")
    if f == 0:
        return "0" if math.copysign(1.0, f) > 0 else "-0"
    a = abs(f)
    if 1e-6 <= a < 1e21:
        r = repr(float(f))
        if "e" in r or "E" in r:  # python switches to exponent earlier (e.g. 1e16)
            r = format(f, "f")
            if "." in r:
                r = r.rstrip("0").rstrip(".")
        elif r.endswith(".0"):
            r = r[:-2]
        return r
    r = repr(float(f))
    mant, _, exp = r.partition("e")
    if mant.endswith(".0"):
        mant = mant[:-2]
    e = int(exp)
    sign = "-" if e < 0 else "+"
    return f"{mant}e{sign}{abs(e):02d}"


def _esc(s: str) -> str:
    out = json.dumps(s, ensure_ascii=False)
    return (out.replace("<", "\\u003c").replace(">", "\\u003e").replace("&", "\\u0026")
            .replace("\u2028", "\\u2028").replace("\u2029", "\\u2029"))


class GoRaw:
    """Pre-encoded JSON fragment."""

    def __init__(self, raw: str):
        self.raw = raw


def dumps(v, sort_dict_keys: bool = True) -> str:
    """Encode. Python dicts are Go *maps* (keys sorted) unless wrapped in
    ``GoStruct`` (ordered fields, like a Go struct)."""
    if isinstance(v, GoRaw):
        return v.raw
    if v is None:
        return "null"
    if v is True:
        return "true"
    if v is False:
        return "false"
    if isinstance(v, int):
        return str(v)
    if isinstance(v, float):
        return go_float(v)
    if isinstance(v, str):
        return _esc(v)
    if isinstance(v, (bytes, bytearray, memoryview)):
        return '"' + base64.b64encode(bytes(v)).decode() + '"'
    if isinstance(v, GoStruct):
        return "{" + ",".join(_esc(k) + ":" + dumps(x) for k, x in v.items) + "}"
    if isinstance(v, dict):
        keys = sorted(v) if sort_dict_keys else list(v)
        return "{" + ",".join(_esc(str(k)) + ":" + dumps(v[k]) for k in keys) + "}"
    if isinstance(v, (list, tuple)):
        return "[" + ",".join(dumps(x) for x in v) + "]"
    raise TypeError(f"cannot encode {type(v)}")


class GoStruct:
    """Ordered (field, value) pairs; ``omitempty`` fields are dropped by the caller."""

    def __init__(self, *items: tuple[str, object]):
        self.items = list(items)


def struct(**fields) -> GoStruct:
    return GoStruct(*fields.items())
