#!/usr/bin/env python3
"""Registers, occupancy and LDS of the hot decode kernels, from the compiler's
resource remarks (``hipcc -Rpass-analysis=kernel-resource-usage``, device-only
compile of ``gemm_skinny.hip`` and ``attn_decode.hip`` for gfx950; ~2 min).

The question it answers: can a Whisper decoder wave sit beside an LLM decode
GEMM workgroup on the same CU (one 512-entry VGPR + AGPR file per SIMD lane)?

    python scripts/kernel_registers.py > profiles/r6_decode_kernel_registers.txt
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
KDIR = os.path.join(ROOT, "csrc", "kernels")

LABELS = {
    "SF<2, 1, 4, 4, 1, 1, 0, 0, 0>": "8B gate|up (SiLU, RMS prologue)",
    "SF<2, 1, 4, 1, 2, 0, 0, 0, 0>": "8B down (+residual)",
    "SF<2, 1, 4, 1, 3, 1, 0, 0, 0>": "8B qkv (RoPE + KV append, RMS)",
    "SF<1, 1, 4, 1, 2, 0, 0, 0, 0>": "8B o (+residual)",
    "SF<1, 1, 2, 1, 2, 0, 0, 0, 0>": "Whisper o / cross-o (+residual)",
    "SF<2, 1, 2, 1, 4, 2, 0, 0, 0>": "Whisper fc1 (GELU, LN)",
    "SF<2, 1, 2, 1, 2, 0, 0, 0, 0>": "Whisper fc2 (+residual)",
    "SF<1, 1, 2, 1, 3, 2, 0, 0, 0>": "Whisper self qkv (LN, KV append)",
    "SF<1, 1, 2, 1, 4, 2, 0, 0, 0>": "Whisper cross q (LN)",
    "SF<2, 1, 4, 1, 1, 1, 0, 0, 0>": "70B shard gate|up",
    "SF<2, 1, 4, 1, 4, 0, 0, 0, 0>": "70B shard o / down (partials)",
    "SF<1, 1, 4, 1, 3, 1, 0, 0, 0>": "70B shard qkv",
    "attn_decode_kernel<128, 0, 4, 2>": "Llama decode attention (D 128)",
    "attn_decode_kernel<64, 0, 4, 2>": "Whisper self / cross attention (D 64)",
}
PAT = {"V": r"VGPRs: (\d+)", "A": r"AGPRs: (\d+)", "occ": r"Occupancy \[waves/SIMD\]: (\d+)",
       "LDS": r"LDS Size \[bytes/block\]: (\d+)", "spill": r"VGPRs Spill: (\d+)"}


def remarks(src: str) -> str:
    with tempfile.TemporaryDirectory() as td:
        r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                            "-munsafe-fp-atomics", "--offload-device-only", f"-I{KDIR}", "-c",
                            os.path.join(KDIR, src), "-o", os.path.join(td, "k.o"),
                            "-Rpass-analysis=kernel-resource-usage"],
                           capture_output=True, text=True)
    if r.returncode:
        sys.exit(r.stderr[-2000:])
    return r.stderr


def main() -> int:
    print("# registers / occupancy of the hot decode kernels (hipcc -O3 --offload-arch=gfx950 "
          "-Rpass-analysis=kernel-resource-usage; scripts/kernel_registers.py)")
    print("# V = arch VGPRs, A = AGPRs (one 512-entry file per SIMD lane); occ = waves per SIMD "
          "of the kernel alone")
    for src in ("gemm_skinny.hip", "attn_decode.hip"):
        blocks = re.split(r"remark: Function Name: ", remarks(src))[1:]
        names = [b.split(" ")[0] for b in blocks]
        dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True,
                             text=True).stdout.split("\n")
        for b, d in zip(blocks, dem):
            d = (d.replace("skinny_fused_kernel", "SF").replace("(FusedArgs)", "")
                 .replace("(AttnDecArgs)", "").replace("void ", "").strip())
            if d in LABELS:
                vals = {k: (m.group(1) if (m := re.search(p, b)) else "?") for k, p in PAT.items()}
                print(f"{LABELS[d]:38s} {d:34s} " + " ".join(f"{k}={v}" for k, v in vals.items()))
    return 0


if __name__ == "__main__":
    sys.exit(main())
