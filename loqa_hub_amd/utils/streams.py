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
    hip = ctypes.CDLL("libamdhip64.so", mode=ctypes.RTLD_GLOBAL)
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


def stream_for(device: torch.device, env_key: str, priority: int = 0):
    """The stream a worker thread should use: CU-masked when ``env_key`` is
    set (e.g. ``LOQA_STT_CUS=0-63``), else a plain stream of ``priority``."""
    spec = os.environ.get(env_key, "")
    if spec:
        n = torch.cuda.get_device_properties(device).multi_processor_count
        return cu_masked_stream(device, parse_cu_spec(spec, n))
    return torch.cuda.Stream(device, priority=priority)


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
