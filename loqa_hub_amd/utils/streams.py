"""CU-masked HIP streams (spatial partitioning of the 256 CUs).

The STT and LLM decoders are two latency-bound kernel chains that share the
GPU. With plain streams the bandwidth-bound LLM GEMMs occupy CU slots that the
Whisper decoder's small kernels then wait for; ``hipExtStreamCreateWithCUMask``
gives a stream (its hardware queue) a fixed subset of CUs, so the two chains
can be spatially partitioned. Graphs replayed on such a stream inherit the mask.

Masks are given as specs: ``"0-63"`` (a range), ``"0-63,128-191"`` (ranges),
``"stride:4:0"`` (every 4th CU starting at 0), ``"~stride:4:0"`` (complement).
"""
from __future__ import annotations

import ctypes
import os

import torch

from .hip_runtime import hip_runtime

N_CUS_DEFAULT = 256


def parse_cu_spec(spec: str, n_cus: int = N_CUS_DEFAULT) -> list[int]:
    spec = spec.strip()
    neg = spec.startswith("~")
    if neg:
        spec = spec[1:]
    cus: set[int] = set()
    if spec.startswith("stride:"):
        _, step, start = spec.split(":")
        cus = set(range(int(start), n_cus, int(step)))
    else:
        for part in spec.split(","):
            part = part.strip()
            if not part:
                continue
            if "-" in part:
                a, b = part.split("-")
                cus.update(range(int(a), int(b) + 1))
            else:
                cus.add(int(part))
    if neg:
        cus = set(range(n_cus)) - cus
    return sorted(c for c in cus if 0 <= c < n_cus)


def cu_mask_words(cus: list[int], n_cus: int = N_CUS_DEFAULT) -> list[int]:
    words = [0] * ((n_cus + 31) // 32)
    for c in cus:
        words[c // 32] |= 1 << (c % 32)
    return words


_keep: list = []


def cu_masked_stream(device: torch.device, cus: list[int]) -> torch.cuda.ExternalStream:
    """A HIP stream restricted to ``cus`` on ``device`` (wrapped for torch)."""
    hip = hip_runtime()
    n = torch.cuda.get_device_properties(device).multi_processor_count
    words = cu_mask_words(cus, max(n, max(cus) + 1 if cus else n))
    arr = (ctypes.c_uint32 * len(words))(*words)
    handle = ctypes.c_void_p()
    with torch.cuda.device(device):
        rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(handle), ctypes.c_uint32(len(words)), arr)
    if rc != 0:
        raise RuntimeError(f"hipExtStreamCreateWithCUMask failed: {rc}")
    _keep.append(handle)
    return torch.cuda.ExternalStream(handle.value, device=device)


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


def _log_slot(role: str, st, device, priority: int) -> None:
    if os.environ.get("LOQA_LOG_STREAMS"):
        print(f"[streams] {role}: priority {priority} pool slot {pool_slot(st, device, priority)}",
              flush=True)


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
DEFAULT_SLOTS = {"llm": 2, "stt": 30, "encoder": 28, "prefill": 3, "tts": 29}


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
    _log_slot(role, st, device, priority)
    return st


def pool_stream(device: torch.device, role: str, priority: int = 0):
    """A worker thread's stream: the explicitly placed pool stream of ``role``
    (``placed_stream``); ``LOQA_POOL_SKEW_<ROLE>`` = n instead draws n extra
    pool streams and takes the next one (the round-2 placement search)."""
    skew = int(os.environ.get(f"LOQA_POOL_SKEW_{role.upper()}", "0") or 0)
    if not skew:
        return placed_stream(device, role, priority)
    for _ in range(skew):
        torch.cuda.Stream(device, priority=priority)
    st = torch.cuda.Stream(device, priority=priority)
    _log_slot(role, st, device, priority)
    return st


_decoders: dict = {}
_dec_lock = __import__("threading").Lock()


def _hip_stream(device: torch.device, priority: int) -> torch.cuda.ExternalStream:
    hip = hip_runtime()
    handle = ctypes.c_void_p()
    with torch.cuda.device(device):
        rc = hip.hipStreamCreateWithPriority(ctypes.byref(handle), ctypes.c_uint(1), ctypes.c_int(priority))
    if rc != 0:
        raise RuntimeError(f"hipStreamCreateWithPriority failed: {rc}")
    _keep.append(handle)
    return torch.cuda.ExternalStream(handle.value, device=device)


def decoder_streams(device: torch.device, priorities: dict) -> dict:
    """The STT and LLM decoder streams, created ONCE per device, in a fixed
    order, by whichever scheduler thread asks first.

    HIP spreads a process's streams over a few hardware queues
    (GPU_MAX_HW_QUEUES, 4 here) in creation order. Which queues the two
    graph-replaying decoder streams share decides how the GPU interleaves
    them, and measured end to end that is worth 11 vs 17 vs 19 utt/s
    (docs/PERF.md, "the 1.8x cliff"). Pool streams (``torch.cuda.Stream()``)
    made the placement depend on how many streams anything else drew first,
    so these are dedicated HIP streams. ``LOQA_QSKEW="a,b"`` creates ``a``
    spacer streams before the STT stream and ``b`` between it and the LLM
    stream. Opt-in (set ``LOQA_QSKEW``): the four placements measured so far
    gave 17.1 / 17.4 / 9.5 / 17.5 utt/s, while the default pool placement
    measures 18.7-19.2."""
    d = torch.device(device)
    key = d.index if d.index is not None else torch.cuda.current_device()
    with _dec_lock:
        if key not in _decoders:
            a, b = (int(t) for t in os.environ.get("LOQA_QSKEW", DEFAULT_QSKEW).split(","))
            spacers = [_hip_stream(d, 0) for _ in range(a)]
            stt = _hip_stream(d, priorities.get("stt", 0))
            spacers += [_hip_stream(d, 0) for _ in range(b)]
            llm = _hip_stream(d, priorities.get("llm", 0))
            _decoders[key] = {"stt": stt, "llm": llm, "spacers": spacers}
        return _decoders[key]


DEFAULT_QSKEW = "0,0"
_ROLE = {"LOQA_STT_CUS": "stt", "LOQA_LLM_CUS": "llm"}
_PRIO: dict = {}


def stream_for(device: torch.device, env_key: str, priority: int = 0):
    """The stream a worker thread should use: CU-masked when ``env_key`` is
    set (e.g. ``LOQA_STT_CUS=0-63``), else the decoder's dedicated stream."""
    spec = os.environ.get(env_key, "")
    if spec:
        n = torch.cuda.get_device_properties(device).multi_processor_count
        return cu_masked_stream(device, parse_cu_spec(spec, n))
    role = _ROLE.get(env_key)
    if role is None or not os.environ.get("LOQA_QSKEW"):
        # default: explicitly placed pool streams (placed_stream);
        # LOQA_POOL_SKEW_STT / _LLM = n draws n pool streams first, moving this
        # decoder n hardware queues along (the round-2 placement search).
        return pool_stream(device, role or env_key, priority)
    _PRIO[role] = priority
    prios = {"stt": _PRIO.get("stt", -1), "llm": _PRIO.get("llm", 0)}
    return decoder_streams(device, prios)[role]


def decode_cus(device: torch.device, cus_env: str, cap_env: str) -> int | None:
    """Workgroup cap for an engine's decode grids: ``cap_env`` if set, else the
    number of CUs its stream is confined to by ``cus_env``, else None (the
    global default). A grid wider than its CU share would run in two rounds."""
    if os.environ.get(cap_env):
        return int(os.environ[cap_env])
    spec = os.environ.get(cus_env, "")
    if spec and torch.device(device).type == "cuda":
        n = torch.cuda.get_device_properties(device).multi_processor_count
        return len(parse_cu_spec(spec, n))
    return None
