"""Whisper-large-v3 decoder step (graph replay, B=4 live) alone vs beside
background load: a bandwidth hog with few workgroups (CU slots free) and a
slot hog (ALU-only workgroups filling CU slots, no memory traffic)."""
import ctypes, json, os, sys, threading, time
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from loqa_hub_amd.engine.stt_engine import STTEngine, STTRequest  # noqa: E402
from loqa_hub_amd.models.configs import whisper_config  # noqa: E402
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libgemv_exp.so"))
vp, ci, cl = ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong
lib.exp_hog_stream.argtypes = [vp, cl, ci, vp, ci, vp]
lib.exp_hog_alu.argtypes = [ci, vp, ci, vp]
dev = torch.device("cuda", 0)
eng = STTEngine(whisper_config("whisper-large-v3"), dev, seed=0, max_batch=8)
rng = np.random.default_rng(0)
reqs = [STTRequest((rng.standard_normal(48000) * 3000).astype(np.int16), max_new_tokens=400) for _ in range(4)]
eng._admit(reqs, [0, 1, 2, 3])
for r in reqs:
    r.feed = [eng.sot[0]]
for _ in range(3):
    eng._step(reqs)            # capture + warm the graph bucket
    for r in reqs:
        r.feed = [eng.sot[0]]
buf = torch.ones(1 << 30, device=dev, dtype=torch.bfloat16)
out = torch.zeros(16, device=dev)
bg_stream = torch.cuda.Stream(dev)
stop = threading.Event()


def background(kind, grid):
    torch.cuda.set_device(dev)
    with torch.cuda.stream(bg_stream):
        while not stop.is_set():
            if kind == "bw":
                lib.exp_hog_stream(buf.data_ptr(), buf.numel() * 2, 1, out.data_ptr(), grid, bg_stream.cuda_stream)
            else:
                lib.exp_hog_alu(200000, out.data_ptr(), grid, bg_stream.cuda_stream)
            bg_stream.synchronize()


def measure(n=20):
    ts = []
    for _ in range(n):
        for r in reqs:
            r.feed = [eng.sot[0]]
        t0 = time.perf_counter()
        eng._step(reqs)
        ts.append((time.perf_counter() - t0) * 1e3)
    return float(np.median(ts))


print(json.dumps({"case": "alone", "ms": round(measure(), 3)}), flush=True)
for kind, grid in (("bw", 64), ("bw", 256), ("bw", 1024), ("alu", 256), ("alu", 1024), ("alu", 2048)):
    stop.clear()
    th = threading.Thread(target=background, args=(kind, grid), daemon=True)
    th.start()
    time.sleep(0.3)
    ms = measure()
    stop.set()
    th.join()
    print(json.dumps({"case": kind, "grid": grid, "ms": round(ms, 3)}), flush=True)
