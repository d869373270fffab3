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

# LLM decode steps: cap a step's tokens at a smaller padded-row bucket when
# that samples more sequences per unit of step cost (plan_step_mpad)
MPAD_PLAN = True


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


# Relative cost of a decode step by its padded row count (Llama-3-8B fused
# decode step, graph-replayed, scripts/exp/step_cost_by_t.py: T = 16 / 32 / 64
# tokens -> 3.31 / 4.09 / 7.44 ms; the weight stream dominates at 16 rows and
# the MFMA tiles at 64).
MPAD_COST = {16: 1.0, 32: 1.24, 64: 2.25, 128: 4.5}


def _mpad(t: int) -> int:
    for p in MPAD_COST:
        if t <= p:
            return p
    return t


def plan_step_mpad(lens: list[int], budget: int, max_q: int, start: int = 0,
                   whole: list[bool] | None = None) -> list[int]:
    """``plan_step``, but a plan whose token count spills into a larger padded
    row bucket is compared with the plan capped at each smaller bucket: the
    plan with the most sequences that SAMPLE this step (fed their whole feed)
    per unit of step cost wins (ties: the larger plan). A capped plan defers
    the tail of a jump-forward literal to the next step - same tokens, one
    step later for that sequence - instead of making every sequence's step
    ~25% slower. ``whole[i]``: sequence i cannot be split (a speculative feed);
    a partial take of it sits the step out."""
    n = len(lens)
    whole = whole or [False] * n

    def effective(take):
        return [0 if (w and t < L) else t for t, L, w in zip(take, lens, whole)]

    def score(take):
        T = sum(take)
        if T == 0:
            return -1.0
        samples = sum(1 for t, L in zip(take, lens) if t and t == L)
        return samples / MPAD_COST.get(_mpad(T), T / 16)

    best = effective(plan_step(lens, budget, max_q, start))
    T = sum(best)
    if T <= 16:
        return best
    best_s = score(best)
    for cap in MPAD_COST:
        if cap >= _mpad(T) or cap > budget:
            break
        cand = effective(plan_step(lens, cap, max_q, start))
        s = score(cand)
        if s > best_s * 1.0001:
            best, best_s = cand, s
    return best
