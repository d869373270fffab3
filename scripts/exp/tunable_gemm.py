"""Prefill / encoder projection GEMMs: hipBLASLt's default heuristic pick vs
the TunableOp-searched solution (every hipBLASLt + rocBLAS candidate timed).

Weights rotate over enough copies to be cold (a real 32-layer pass never
re-reads a layer's weights), as in gemm_cold_bench.py. Prints one JSON line
per shape: default us, tuned us, and the tuned solution name."""
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

dev = torch.device("cuda", 0)
OUT = os.environ.get("TUNE_FILE", "gpurun_out/tunableop_exp.csv")
SHAPES = [
    # (tag, M, N, K)   Llama-3-8B prefill of one ~318-token parser prompt
    ("llm_qkv", 320, 6144, 4096), ("llm_o", 320, 4096, 4096),
    ("llm_gate_up", 320, 28672, 4096), ("llm_down", 320, 4096, 14336),
    # Whisper-large-v3 encoder, one and four 30-s windows
    ("enc_qkv_b1", 1500, 3840, 1280), ("enc_o_b1", 1500, 1280, 1280),
    ("enc_fc1_b1", 1500, 5120, 1280), ("enc_fc2_b1", 1500, 1280, 5120),
    ("enc_qkv_b4", 6000, 3840, 1280), ("enc_fc2_b4", 6000, 1280, 5120),
]
ONLY = os.environ.get("ONLY")


def timed(x, ws, reps=40):
    for w in ws[:2]:
        F.linear(x, w)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for i in range(reps):
        F.linear(x, ws[i % len(ws)])
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) * 1e3 / reps


def main():
    torch.manual_seed(0)
    res = {}
    data = {}
    for tag, M, N, K in SHAPES:
        if ONLY and tag not in ONLY.split(","):
            continue
        nw = max(2, min(16, int(1.2e9 // (N * K * 2))))
        ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(nw)]
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        data[tag] = (x, ws)
        res[tag] = {"M": M, "N": N, "K": K, "default_us": round(timed(x, ws), 2)}
        print(f"default {tag} {res[tag]['default_us']}", flush=True)
    import torch.cuda.tunable as tun
    tun.enable(True)
    tun.tuning_enable(True)
    tun.set_filename(OUT, insert_device_ordinal=False)
    tun.set_max_tuning_duration(int(os.environ.get("TUNE_MS", "40")))
    tun.set_max_tuning_iterations(int(os.environ.get("TUNE_IT", "20")))
    for tag, (x, ws) in data.items():
        t0 = time.perf_counter()
        F.linear(x, ws[0])
        torch.cuda.synchronize()
        res[tag]["tune_s"] = round(time.perf_counter() - t0, 1)
        print(f"tuned {tag} in {res[tag]['tune_s']} s", flush=True)
    tun.tuning_enable(False)
    for tag, (x, ws) in data.items():
        res[tag]["tuned_us"] = round(timed(x, ws), 2)
    tun.write_file()
    sols = {}
    for r in tun.get_results():
        sols[(r[1])] = r[2]
    for tag, r in res.items():
        M, N, K = r["M"], r["N"], r["K"]
        r["solution"] = next((v for k, v in sols.items() if f"{M}" in k and f"{N}" in k and f"{K}" in k), None)
        print(json.dumps({"tag": tag, **r}), flush=True)


if __name__ == "__main__":
    sys.exit(main())
