"""Whisper decoder step (B=4) alone vs beside the REAL Llama-3-8B decode loop
(graph replay, B=8) and beside the Whisper encoder; and the Llama step alone
vs beside the Whisper decoder loop."""
import json, os, sys, threading, time
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from loqa_hub_amd.engine.llm_engine import GenRequest, LLMEngine  # noqa: E402
from loqa_hub_amd.engine.grammar import multi_command_schema  # noqa: E402
from loqa_hub_amd.engine.stt_engine import STTEngine, STTRequest  # noqa: E402
from loqa_hub_amd.models.configs import llama_config, whisper_config  # noqa: E402
dev = torch.device("cuda", 0)
stt = STTEngine(whisper_config("whisper-large-v3"), dev, seed=0, max_batch=8)
llm = LLMEngine(llama_config("llama3-8b"), dev, seed=0, max_seqs=8, max_seq_len=1024)
stt.warmup_graphs(); llm.warmup_graphs()
rng = np.random.default_rng(0)
sreqs = [STTRequest((rng.standard_normal(48000) * 3000).astype(np.int16), max_new_tokens=400) for _ in range(4)]
stt._admit(sreqs, [0, 1, 2, 3])
lreqs = [GenRequest(list(range(5, 300)), multi_command_schema(8, min_response_tokens=200, max_response_tokens=400))
         for _ in range(8)]
for r in lreqs:
    llm.submit(r)
llm.prefill(lreqs)


def stt_step():
    for r in sreqs:
        r.feed = [stt.sot[0]]
    stt._step(sreqs)


def llm_step():
    llm.decode_step([r for r in lreqs if not r.done])


def timed(fn, n=30):
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        ts.append((time.perf_counter() - t0) * 1e3)
    return float(np.median(ts))


stop = threading.Event()


def bg(fn, stream):
    torch.cuda.set_device(dev)
    torch.cuda.set_stream(stream)
    while not stop.is_set():
        fn()


def encode_loop():
    audio = torch.zeros(2, 480000, device=dev)
    with torch.inference_mode():
        stt.model.encode(audio)
    torch.cuda.current_stream().synchronize()


def with_bg(fg, bgfn):
    stop.clear()
    s = torch.cuda.Stream(dev)
    th = threading.Thread(target=bg, args=(bgfn, s), daemon=True)
    th.start()
    time.sleep(0.3)
    ms = timed(fg)
    stop.set()
    th.join()
    return ms


torch.cuda.set_stream(torch.cuda.Stream(dev))
res = {"stt_alone": timed(stt_step), "llm_alone": timed(llm_step)}
res["stt_with_llm"] = with_bg(stt_step, llm_step)
res["llm_with_stt"] = with_bg(llm_step, stt_step)
res["stt_with_encoder"] = with_bg(stt_step, encode_loop)
res["llm_with_encoder"] = with_bg(llm_step, encode_loop)
print(json.dumps({k: round(v, 3) for k, v in res.items()}), flush=True)
