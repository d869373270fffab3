"""Which LLM decode kernel slows the concurrent Whisper decoder step?
Background loops of one kernel type each (Llama-3-8B shapes, B=8 decode)."""
import json, os, sys, threading, time
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from loqa_hub_amd import ops  # noqa: E402
from loqa_hub_amd.engine.stt_engine import STTEngine, STTRequest  # noqa: E402
from loqa_hub_amd.models.configs import whisper_config  # noqa: E402
dev = torch.device("cuda", 0)
stt = STTEngine(whisper_config("whisper-large-v3"), dev, seed=0, max_batch=8)
stt.warmup_graphs()
rng = np.random.default_rng(0)
sreqs = [STTRequest((rng.standard_normal(48000) * 3000).astype(np.int16), max_new_tokens=400) for _ in range(4)]
stt._admit(sreqs, [0, 1, 2, 3])


def stt_step():
    for r in sreqs:
        r.feed = [stt.sot[0]]
    stt._step(sreqs)


def timed(fn, n=30):
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        ts.append((time.perf_counter() - t0) * 1e3)
    return float(np.median(ts))


bf = dict(device=dev, dtype=torch.bfloat16)
scr = ops.FusedScratch(dev)
M = 16
x = torch.randn(M, 4096, **bf)
ws = {n: [ops.shuffle_weight(torch.randn(N, K, **bf) * 0.02) for _ in range(c)]
      for n, N, K, c in (("gate_up", 28672, 4096, 3), ("down", 4096, 14336, 6), ("o", 4096, 4096, 16),
                         ("lm", 128256, 4096, 1))}
xd = torch.randn(M, 14336, **bf)
res = torch.randn(M, 4096, **bf)
scr.rowsq[: 128 * M].fill_(32.0)
H, Hkv, D, blk, B, ctx = 32, 8, 128, 16, 8, 500
nb = B * 64
kc = torch.randn(nb, Hkv, blk, D, **bf)
vc = torch.randn_like(kc)
bt = torch.arange(nb, dtype=torch.int32, device=dev).view(B, -1)
q = torch.randn(16, H * D, **bf)
cu = torch.arange(B + 1, dtype=torch.int32, device=dev)
cl = torch.full((B,), ctx, dtype=torch.int32, device=dev)
aws = ops.AttnWorkspace(dev, 256, H, D, 32)
it = iter(range(1 << 40))
def gu(S, rt, wr):
    return lambda: ops.skinny_fused(x, ws["gate_up"][next(it) % 3], "silu", scr, splits=S, rt=rt, wr=wr,
                                    norm=True, rowsq_tiles=128)


def dn(S, rt, wr):
    return lambda: ops.skinny_fused(xd, ws["down"][next(it) % 6], "resid", scr, splits=S, rt=rt, wr=wr,
                                    residual=res)


kernels = {
    "gu_S1rt2wr4": gu(1, 2, 4), "gu_S1rt1wr4": gu(1, 1, 4), "gu_S1rt2wr1": gu(1, 2, 1),
    "gu_S2rt2wr1": gu(2, 2, 1), "gu_S1rt1wr1": gu(1, 1, 1),
    "dn_S2rt2wr1": dn(2, 2, 1), "dn_S1rt1wr1": dn(1, 1, 1), "dn_S1rt2wr1": dn(1, 2, 1),
}
stop = threading.Event()


def bg(fn, stream):
    torch.cuda.set_device(dev)
    torch.cuda.set_stream(stream)
    g = torch.cuda.CUDAGraph()
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        for _ in range(20):
            fn()
    while not stop.is_set():
        g.replay()
        stream.synchronize()


sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench_kernels import gtime  # noqa: E402
alone = {n: round(gtime(f, inner=24), 2) for n, f in kernels.items()}
print(json.dumps({"kernel_alone_us": alone}), flush=True)
torch.cuda.set_stream(torch.cuda.Stream(dev))
out = {"stt_alone": timed(stt_step)}
for name, fn in kernels.items():
    stop.clear()
    s = torch.cuda.Stream(dev)
    th = threading.Thread(target=bg, args=(fn, s), daemon=True)
    th.start()
    time.sleep(0.5)
    out[name] = timed(stt_step)
    stop.set()
    th.join()
print(json.dumps({k: round(v, 3) for k, v in out.items()}), flush=True)
