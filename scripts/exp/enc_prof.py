"""Isolated Whisper-large-v3 front end + encoder + cross-K/V projection per
batch size (the STT admission work of one arrival micro-batch)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from loqa_hub_amd.engine.stt_engine import STTEngine, STTRequest  # noqa: E402
from loqa_hub_amd.engine.synthetic import make_unique  # noqa: E402
from loqa_hub_amd.models.configs import whisper_config  # noqa: E402

dev = torch.device("cuda", 0)
print("init", flush=True)
eng = STTEngine(whisper_config(os.environ.get("MODEL", "whisper-large-v3")), dev, seed=0, max_batch=8)
utts = make_unique(0, [2] * 16)
out = {}
BS = [int(b) for b in os.environ.get("ENC_BS", "1,2,4").split(",")]
ITERS = int(os.environ.get("ENC_ITERS", "6"))
for B in BS:
    reqs = [STTRequest(u.pcm, transcript=u.text) for u in utts[:B]]
    ts = []
    for it in range(ITERS):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng._encode(reqs, list(range(B)))
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
        print(f"B{B} it{it} {ts[-1] * 1e3:.2f} ms", flush=True)
    ts = sorted(ts[2:])
    out[f"B{B}_ms"] = round(ts[len(ts) // 2] * 1e3, 2)
print(json.dumps(out), flush=True)
