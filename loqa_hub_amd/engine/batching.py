"""Per-step token budgeting shared by the STT and LLM continuous-batching
schedulers.

A decode step feeds each live sequence a few tokens: the LLM its sampled token
plus the grammar's jump-forward literal (``LLMEngine.decode_step``), a new
Whisper sequence its 4-token start-of-transcript prompt. The fused decode
GEMMs and the captured graphs are sized for at most ``ops.MPADS`` rows, so the
step's TOTAL token count must stay under a budget however many sequences are
live. ``plan_step`` splits the budget:

1. one token for every sequence, in round-robin order from ``start`` (so
   when more sequences are live than the budget allows, the ones left out
   this step go first next step);
2. the rest of the budget tops sequences up to ``min(len(feed), max_q)``,
   in the same order.

A sequence fed less than its whole feed "carries" the remainder to the next
step (its logits that step are unused), exactly like a forced literal longer
than ``max_q``.
"""
from __future__ import annotations

import threading
from concurrent.futures import Future


def join_futures(parts: list[Future], result) -> Future:
    """One future over ``parts``: resolves with ``result`` when all succeed,
    fails with the first part's exception."""
    fut: Future = Future()
    left = [len(parts)]
    lock = threading.Lock()

    def _part_done(f: Future) -> None:
        with lock:
            left[0] -= 1
            if fut.done():
                return
            if f.exception() is not None:
                fut.set_exception(f.exception())
            elif left[0] == 0:
                fut.set_result(result)
    for p in parts:
        p.add_done_callback(_part_done)
    return fut


def plan_step(lens: list[int], budget: int, max_q: int, start: int = 0) -> list[int]:
    """Tokens to feed each sequence this step (0 = sits the step out)."""
    n = len(lens)
    take = [0] * n
    if n == 0:
        return take
    budget = max(1, budget)
    order = [(start + i) % n for i in range(n)]
    left = budget
    for i in order:
        if left == 0:
            break
        if lens[i] > 0:
            take[i] = 1
            left -= 1
    for i in order:
        if left == 0:
            break
        if take[i]:
            extra = min(lens[i], max_q) - 1
            if extra > 0:
                e = min(extra, left)
                take[i] += e
                left -= e
    return take
