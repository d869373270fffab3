"""Fault injection (SURVEY §5.3 "New": env ``FAULT_INJECT``).

The reference has no chaos tooling; its recovery paths (STT failure -> error
reply ``audio_service.go:764-815``, TTS graceful degrade ``:182-195``,
compound -> single-parse fallback ``command_parser.go:342-372``, queue rollback
``command_queue.go:132-143``) are only exercised by mocks. Here every
recovery path can be driven on a live hub:

    FAULT_INJECT="stt_error,llm_timeout,tts_error,gpu_kill:1,nats_down"

Entries are separated by ``,`` or ``|``; an entry may carry an argument after
``:`` (``gpu_kill:<rank>`` kills that DP worker; ``gpu_kill:<rank>@<n>`` after
its n-th request) and an optional probability suffix ``%p`` (``stt_error%0.1``
fails 10 % of utterances, drawn from a seeded RNG so runs are reproducible).
"""
from __future__ import annotations

import os
import random
import threading

KNOWN = ("stt_error", "llm_timeout", "tts_error", "gpu_kill", "nats_down")


class InjectedFault(RuntimeError):
    """Raised at an injection site; carries the fault name."""

    def __init__(self, name: str):
        super().__init__(f"injected fault: {name}")
        self.fault = name


class FaultInjector:
    def __init__(self, spec: str | None = None, seed: int = 0):
        spec = os.environ.get("FAULT_INJECT", "") if spec is None else spec
        self.entries: dict[str, tuple[str | None, float]] = {}
        for raw in spec.replace("|", ",").split(","):
            raw = raw.strip()
            if not raw:
                continue
            prob = 1.0
            if "%" in raw:
                raw, p = raw.split("%", 1)
                prob = float(p)
            name, _, arg = raw.partition(":")
            if name not in KNOWN:
                raise ValueError(f"unknown fault {name!r} (known: {', '.join(KNOWN)})")
            self.entries[name] = (arg or None, prob)
        self._rng = random.Random(seed)
        self._lock = threading.Lock()
        self.fired: dict[str, int] = {}

    def __bool__(self) -> bool:
        return bool(self.entries)

    def arg(self, name: str) -> str | None:
        e = self.entries.get(name)
        return e[0] if e else None

    def active(self, name: str) -> bool:
        """True when ``name`` is configured and its probability draw fires."""
        e = self.entries.get(name)
        if e is None:
            return False
        with self._lock:
            hit = e[1] >= 1.0 or self._rng.random() < e[1]
            if hit:
                self.fired[name] = self.fired.get(name, 0) + 1
        return hit

    def check(self, name: str) -> None:
        if self.active(name):
            raise InjectedFault(name)

    def gpu_kill_after(self, rank: int) -> int | None:
        """Requests after which DP worker ``rank`` dies (None: never)."""
        a = self.arg("gpu_kill")
        if a is None:
            return None
        r, _, n = a.partition("@")
        if int(r) != rank:
            return None
        return int(n) if n else 1


_global: FaultInjector | None = None


def faults() -> FaultInjector:
    """Process-wide injector built from ``FAULT_INJECT`` on first use."""
    global _global
    if _global is None:
        _global = FaultInjector()
    return _global


def set_faults(spec: str | None) -> FaultInjector:
    """Replace the process-wide injector (tests, DP workers)."""
    global _global
    _global = FaultInjector(spec or "")
    return _global
