"""Serving-stream placement on HIP hardware queues.

HIP gives a process a few hardware queues (``GPU_MAX_HW_QUEUES``, 4) and maps
streams onto them in creation order, so which queues the graph-replaying
decoder streams share decides how the GPU interleaves them (measured: 11 vs 19
utt/s, docs/PERF.md "the 1.8x cliff"). Every serving stream is therefore the
PyTorch pool stream at a FIXED index, with both pools created first thing.

Round 4 removed the placement experiments that lost (CU-masked streams,
dedicated spacer streams, pool skews, per-engine priorities; docs/PERF.md).
"""
from __future__ import annotations

import os

import torch

# ---------------------------------------------------------------- pool slots
# PyTorch hands out pool streams round-robin (32 per priority); HIP places a
# process's streams on its few hardware queues by creation order, so a pool
# stream's INDEX decides its hardware queue. Which queues the decoder streams
# share is worth 11 vs 19 utt/s (docs/PERF.md, "the 1.8x cliff"), and before
# this the index a decoder got depended on how many pool streams the tuner had
# drawn first. ``pool_slot`` identifies a pool stream's index from its handle;
# ``aligned_pool_stream`` draws streams until the next one has a given index.
POOL_SIZE = 32
_POOL_TABLES: dict = {}


def _pool_table(device: torch.device, priority: int) -> list[int]:
    d = torch.device(device)
    key = (d.index if d.index is not None else torch.cuda.current_device(), priority)
    tab = _POOL_TABLES.get(key)
    if tab is None:
        # one full cycle of the pool: the cursor ends where it started
        tab = [torch.cuda.Stream(d, priority=priority).cuda_stream for _ in range(POOL_SIZE)]
        _POOL_TABLES[key] = tab
    return tab


def pool_slot(stream, device: torch.device, priority: int) -> int:
    tab = _pool_table(device, priority)
    try:
        return tab.index(stream.cuda_stream)
    except ValueError:
        return -1


def aligned_pool_stream(device: torch.device, priority: int, slot: int):
    """The pool stream with index ``slot`` (mod 32) of this priority's pool."""
    tab = _pool_table(device, priority)
    for _ in range(POOL_SIZE + 1):
        st = torch.cuda.Stream(device, priority=priority)
        if tab.index(st.cuda_stream) == slot % POOL_SIZE:
            return st
    raise RuntimeError("pool stream slot not found")


# Explicit placement: every serving stream is the pool stream of a FIXED index
# (its hardware queue follows from the index), whatever else drew pool streams
# before. Defaults = the placement measured best (docs/PERF.md, "Stream
# placement, round 3"; profiles/r3_stream_placement.txt): the LLM decoder on
# normal-priority slot 2, the Whisper decoder on high-priority slot 30, the
# encoder worker on normal-priority slot 28, the prefill worker on slot 3
# (pools created first thing by init_pools, so slot -> queue is fixed); VITS
# (progressive reply speech) on normal-priority slot 29.
# Round 3 found the old
# implicit placement had depended on the STT upload drawing one pool stream per
# batch: removing that draw moved the LLM decoder to slot 0 and halved the
# throughput (19.1 -> 9.8 utt/s). LOQA_SLOT_<ROLE> overrides (search).
# The PCM stream-in copies (engine/pcm_staging.py) take the old prefill
# worker's slot 3: a queue of their own beside the decoders (the copies run on
# the DMA engine and hold no CU).
DEFAULT_SLOTS = {"llm": 2, "stt": 30, "encoder": 28, "prefill": 3, "tts": 29, "h2d": 3}


def init_pools(device: torch.device) -> None:
    """Create both PyTorch stream pools (normal and high priority) of ``device``
    in one go, before the engines create anything else, so pool index ->
    creation order -> hardware queue is the same in every process that runs
    this code (the engines call it first thing)."""
    if torch.device(device).type != "cuda":
        return
    _pool_table(device, 0)
    _pool_table(device, -1)


def role_slot(role: str) -> int | None:
    v = os.environ.get(f"LOQA_SLOT_{role.upper()}")
    if v is not None:
        return int(v) if v != "" and int(v) >= 0 else None
    return DEFAULT_SLOTS.get(role)


def placed_stream(device: torch.device, role: str, priority: int = 0):
    """The serving stream of ``role``: the pool stream at its fixed slot
    (``LOQA_SLOT_<ROLE>`` = -1: the next pool stream, the old behaviour)."""
    slot = role_slot(role)
    if slot is None:
        st = torch.cuda.Stream(device, priority=priority)
    else:
        st = aligned_pool_stream(device, priority, slot)
    return st


def decode_cap(cap_env: str) -> int | None:
    """Workgroup cap for an engine's decode grids (``cap_env``), else None
    (the global ``LOQA_MAX_DECODE_WGS`` default)."""
    v = os.environ.get(cap_env)
    return int(v) if v else None
