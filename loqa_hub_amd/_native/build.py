"""Build the native HIP/C++ libraries in-tree for gfx950.

Two shared objects are produced next to this file:

* ``libloqa_kernels.so`` - every hand-written CDNA4 kernel under ``csrc/kernels``
  (compiled with ``hipcc --offload-arch=gfx950``).
* ``libloqa_runtime.so`` - the host runtime under ``csrc/runtime`` (pinned PCM
  staging, paged-KV block pool).

They are loaded with ctypes *after* ``import torch`` so the process shares
torch's single HIP runtime (both link ``libamdhip64.so.7``).

Usage: ``python -m loqa_hub_amd._native.build [--force] [--debug]``.
"""
from __future__ import annotations

import argparse
import glob
import hashlib
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
CSRC = os.path.join(REPO, "csrc")
ARCH = os.environ.get("LOQA_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm is required to build the native kernels)")


def _digest(paths: list[str], flags: list[str]) -> str:
    h = hashlib.sha256()
    for p in sorted(paths):
        with open(p, "rb") as f:
            h.update(f.read())
    h.update(" ".join(flags).encode())
    return h.hexdigest()


def _build_lib(name: str, sources: list[str], headers: list[str], flags: list[str],
               force: bool) -> str:
    out = os.path.join(HERE, name)
    stamp = out + ".sha256"
    digest = _digest(sources + headers, flags)
    if not force and os.path.exists(out) and os.path.exists(stamp):
        with open(stamp) as f:
            if f.read().strip() == digest:
                return out
    hipcc = _hipcc()
    objdir = os.path.join(HERE, "build", name)
    os.makedirs(objdir, exist_ok=True)

    def compile_one(src: str) -> str:
        obj = os.path.join(objdir, os.path.basename(src) + ".o")
        cmd = [hipcc, *flags, "-fPIC", "-c", src, "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        return obj

    with ThreadPoolExecutor(max_workers=min(8, len(sources))) as ex:
        objs = list(ex.map(compile_one, sources))
    # link next to the target and rename over it: a reader (a running process,
    # a tree snapshot) never sees a half-written library
    tmp = out + ".tmp"
    cmd = [hipcc, *flags, "-shared", "-fPIC", *objs, "-o", tmp]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, out)
    with open(stamp, "w") as f:
        f.write(digest)
    return out


def build(force: bool = False, debug: bool = False) -> list[str]:
    opt = ["-O0", "-g"] if debug else ["-O3"]
    kflags = [f"--offload-arch={ARCH}", *opt, "-std=c++17", "-munsafe-fp-atomics",
              f"-I{os.path.join(CSRC, 'kernels')}"]
    ksrc = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    khdr = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.h")))
    rsrc = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    rhdr = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.h")))
    rflags = [*opt, "-std=c++17", "-D__HIP_PLATFORM_AMD__"]
    return [
        _build_lib("libloqa_kernels.so", ksrc, khdr, kflags, force),
        _build_lib("libloqa_runtime.so", rsrc, rhdr, rflags, force),
    ]


def build_sanitized(kind: str = "address,undefined", out_dir: str | None = None) -> str:
    """Host-only sanitizer build of the C++ runtime + its stress test
    (GPU sanitizers are not available on the target pool).
    ``kind``: "address,undefined" or "thread". Returns the executable path."""
    out_dir = out_dir or os.path.join(HERE, "build", "sanitize")
    os.makedirs(out_dir, exist_ok=True)
    exe = os.path.join(out_dir, "pool_stress_" + kind.replace(",", "_"))
    cxx = shutil.which("g++") or shutil.which("c++")
    if cxx is None:
        raise RuntimeError("no host C++ compiler")
    cmd = [cxx, "-std=c++17", "-O1", "-g", f"-fsanitize={kind}", "-fno-omit-frame-pointer",
           "-I/opt/rocm/include", "-D__HIP_PLATFORM_AMD__", "-Wno-unused-result",
           os.path.join(CSRC, "runtime", "runtime.cpp"), os.path.join(CSRC, "runtime", "tp_control.cpp"),
           os.path.join(CSRC, "runtime", "tests", "pool_stress.cpp"),
           "-L/opt/rocm/lib", "-lamdhip64", "-lpthread", "-Wl,-rpath,/opt/rocm/lib", "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"sanitizer build failed: {' '.join(cmd)}\n{r.stderr[-3000:]}")
    return exe


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("--sanitize", choices=["address,undefined", "thread"],
                    help="build + run the host runtime stress test under a sanitizer")
    a = ap.parse_args(argv)
    if a.sanitize:
        exe = build_sanitized(a.sanitize)
        return subprocess.run([exe]).returncode
    for p in build(force=a.force, debug=a.debug):
        print(p)
    return 0


if __name__ == "__main__":
    sys.exit(main())
