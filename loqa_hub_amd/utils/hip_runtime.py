"""The HIP runtime this process already uses, for the few direct ctypes calls
(CU-masked / prioritised streams, device flags).

torch links its own ``libamdhip64``; loading the library again by soname could
map a second copy whose state (devices, streams, flags) torch never sees.
``hip_runtime()`` instead resolves the copy already mapped into the process and
opens it with RTLD_NOLOAD, so it can never load anything new.
"""
from __future__ import annotations

import ctypes
import functools
import os


def mapped_hip_path() -> str:
    """Path of the libamdhip64 mapped into this process (torch's)."""
    with open("/proc/self/maps") as f:
        for line in f:
            if "libamdhip64.so" in line:
                return line.split()[-1]
    raise RuntimeError("libamdhip64 is not mapped (import torch first)")


@functools.lru_cache(maxsize=1)
def hip_runtime() -> ctypes.CDLL:
    import torch  # noqa: F401  (torch's HIP libraries link, and so map, libamdhip64)
    return ctypes.CDLL(mapped_hip_path(), mode=os.RTLD_NOLOAD | os.RTLD_GLOBAL)
