"""GIL hand-off latency for the serving threads.

One process drives a GPU from several Python threads: the STT and LLM decode
schedulers, the encoder and prefill workers, and the asyncio control plane.
A scheduler thread that wakes from its step's device read-back must re-take
the GIL before it can launch the next step; while another thread runs Python
code, CPython only forces a hand-off after ``sys.getswitchinterval()`` (5 ms
by default) - a whole decode step of idle GPU. ``tune_switch_interval``
shortens that interval (``LOQA_SWITCH_INTERVAL`` seconds) once per process.
"""
from __future__ import annotations

import os
import sys

_done = False


def tune_switch_interval(default: float | None = None) -> float:
    global _done
    if not _done:
        _done = True
        v = os.environ.get("LOQA_SWITCH_INTERVAL")
        val = float(v) if v else default
        if val is not None and val > 0:
            sys.setswitchinterval(val)
    return sys.getswitchinterval()
