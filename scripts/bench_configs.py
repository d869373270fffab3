#!/usr/bin/env python3
"""The other BASELINE.json configs on ONE MI355X (bench.py measures config 4).

  --config 2  Whisper-base + TinyLlama-1.1B, single utterance at a time (one
              closed-loop stream): per-utterance latency, STT / LLM split and
              ms per added command (marginal over 1-4 command utterances).
  --config 3  Llama-3-8B streaming token decode + multi-command queue with
              rollback, TP=1: text utterances straight into the constrained
              decode; first-token latency, streamed tokens/s, ms per added
              command; every 4th utterance runs with NATS publishes failing
              at random (p = 0.5) so the queue's rollback path executes.
  --config 5  Whisper-large-v3 + Llama-3-70B + VITS TTS of every reply, on ONE
              GPU at TP=1: compact single-copy weights (fused decode layout,
              chunked fused prefill), so 70B bf16 = 141 GB fits in 288 GB
              HBM3E (the TP=8 path is exercised by tests/test_tp.py): 8
              closed-loop streams, utterances/s, ms per added command, TTS
              time per reply.

Synthetic speech-like audio, random-init weights (teacher-forced STT,
grammar-constrained LLM) as in bench.py. Prints one JSON line per config.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from loqa_hub_amd import ops  # noqa: E402
from loqa_hub_amd.engine.llm_engine import LLMEngine  # noqa: E402
from loqa_hub_amd.engine.pipeline import PipelineJob, VoicePipeline, added_command_stats  # noqa: E402
from loqa_hub_amd.engine.stt_engine import STTEngine  # noqa: E402
from loqa_hub_amd.engine.synthetic import make_batch  # noqa: E402
from loqa_hub_amd.llm.transcriber import to_transcription_result  # noqa: E402
from loqa_hub_amd.models.configs import llama_config, vits_config, whisper_config  # noqa: E402


def _closed_loop(pipe, utts, streams: int, per_stream: int, tts=None):
    """``streams`` closed-loop clients, ``per_stream`` utterances each;
    returns (jobs, wall seconds, per-job TTS seconds)."""
    jobs, tts_s = [], []

    async def client(ci):
        for k in range(per_stream):
            u = utts[(ci * per_stream + k) % len(utts)]
            j = PipelineJob(u.relay_id, f"c{ci}-{k}", u.pcm, transcript_hint=u.text)
            await pipe.submit(j)
            if tts is not None and j.multi is not None and j.multi.combined_response:
                t0 = time.perf_counter()
                await tts.synthesize(j.multi.combined_response)
                tts_s.append(time.perf_counter() - t0)
                j.t["tts_done"] = time.perf_counter()
            jobs.append(j)

    async def main():
        t0 = time.perf_counter()
        await asyncio.gather(*[client(c) for c in range(streams)])
        return time.perf_counter() - t0
    wall = asyncio.get_event_loop().run_until_complete(main())
    return jobs, wall, tts_s


def _lat(jobs, key="queue_done"):
    return [(j.t[key] - j.t["start"]) * 1e3 for j in jobs if key in j.t]


def config_2_or_5(cfg_id: int, args, dev, nats) -> dict:
    if cfg_id == 2:
        stt_name, llm_name, streams = "whisper-base", "tinyllama", 1
    else:
        stt_name, llm_name, streams = "whisper-large-v3", "llama3-70b", 8
    t0 = time.perf_counter()
    stt = STTEngine(whisper_config(stt_name), dev, seed=0, max_batch=8)
    # 70B at TP=1: one weight copy in the fused decode layout (141 GB)
    llm = LLMEngine(llama_config(llm_name), dev, seed=0, max_seqs=8, max_seq_len=1024,
                    compact=llm_name == "llama3-70b")
    pipe = VoicePipeline(stt, llm, nats, min_response_tokens=8, max_batch=8)
    pipe.warmup()
    tts = None
    if cfg_id == 5:
        from loqa_hub_amd.engine.tts_engine import VitsTTSEngine
        tts = VitsTTSEngine(vits_config("vits-ljs"), dev, seed=0)
    init_s = time.perf_counter() - t0
    utts = make_batch(0, 16, [1, 2, 3, 4])
    _closed_loop(pipe, utts, streams, args.warmup, tts)           # warm-up
    s0 = dict(llm.stats)
    per_stream = args.per_stream * (4 if streams == 1 else 1)
    jobs, wall, tts_s = _closed_loop(pipe, utts, streams, per_stream, tts)
    st = added_command_stats(jobs)
    lat = _lat(jobs, "tts_done" if tts is not None else "queue_done")
    stt_ms = [(j.t["stt_done"] - j.t["start"]) * 1e3 for j in jobs]
    steps = llm.stats["decode_steps"] - s0["decode_steps"]
    return {
        "config": cfg_id, "model": f"{stt_name} + {llm_name}" + (" + vits-ljs" if tts else ""),
        "n_gpus": 1, "tp": 1, "streams": streams, "utterances": len(jobs), "dtype": "bf16",
        "utterances_per_s": round(len(jobs) / wall, 3),
        "latency_ms_p50": round(float(np.median(lat)), 1),
        "latency_ms_p90": round(float(np.percentile(lat, 90)), 1),
        "stt_ms_mean": round(float(np.mean(stt_ms)), 1),
        "ms_per_added_command_e2e_marginal": None if st["e2e_marginal_ms_per_added_command"] is None
        else round(st["e2e_marginal_ms_per_added_command"], 2),
        "ms_per_added_command_ref_equiv": st["ref_equiv_ms_per_added_command"],
        "llm_ms_per_decode_step": round((llm.stats["decode_s"] - s0["decode_s"]) / max(1, steps) * 1e3, 3),
        "tts_ms_mean": round(float(np.mean(tts_s)) * 1e3, 1) if tts_s else None,
        "command_count_match": float(np.mean([j.n_commands == j.n_expected for j in jobs])),
        "init_s": round(init_s, 1),
        "fused_gemm_tuning": {f"{k[0]}:{k[1]}x{k[2]}:M{k[3]}": list(v) for k, v in ops._FSPLITS.items()},
        "data": "synthetic speech-like PCM16 + random-init weights (teacher-forced STT)",
    }


def config_3(args, dev, nats) -> dict:
    """Text-in streaming decode (no STT): the LLM engine's scheduler thread,
    one stream at a time so first-token latency is unloaded."""
    from loqa_hub_amd.utils.faults import set_faults
    llm = LLMEngine(llama_config("llama3-8b"), dev, seed=0, max_seqs=8, max_seq_len=1024)
    llm.warmup_graphs()
    loop = asyncio.get_event_loop()
    pipe = VoicePipeline(STTEngine.__new__(STTEngine), llm, nats, min_response_tokens=8)
    utts = make_batch(3, 16, [1, 2, 3, 4])
    rows, rollbacks = [], 0

    async def one(i, u):
        nonlocal rollbacks
        j = PipelineJob(u.relay_id, f"t{i}", u.pcm, transcript_hint=u.text)
        j.t["start"] = time.perf_counter()
        j.transcription = to_transcription_result(u.text.split(" ", 2)[-1] if u.text.startswith("hey loqa")
                                                  else u.text)
        toks = []
        j.on_tokens = lambda ids: toks.append((time.perf_counter(), len(ids)))
        fault = i % 4 == 3
        set_faults("nats_down%0.5" if fault else "")
        await pipe._llm_stage([j])
        set_faults("")
        if fault and j.queue is not None and j.queue.rollback_occurred:
            rollbacks += 1
        t_first = toks[1][0] if len(toks) > 1 else toks[0][0]
        n_tok = sum(n for _, n in toks)
        dur = toks[-1][0] - toks[0][0]
        rows.append((j, (t_first - j.t["start"]) * 1e3, n_tok / max(dur, 1e-9)))

    async def main():
        for i, u in enumerate(utts[:4]):
            await one(i, u)             # warm-up
        rows.clear()
        for k in range(args.per_stream * 4):
            await one(k, utts[k % len(utts)])
    loop.run_until_complete(main())
    jobs = [r[0] for r in rows]
    st = added_command_stats(jobs)
    llm.stop()
    return {
        "config": 3, "model": "llama3-8b", "n_gpus": 1, "tp": 1, "dtype": "bf16",
        "utterances": len(jobs),
        "first_token_ms_p50": round(float(np.median([r[1] for r in rows])), 2),
        "stream_tokens_per_s_p50": round(float(np.median([r[2] for r in rows])), 1),
        "ms_per_added_command_e2e_marginal": None if st["e2e_marginal_ms_per_added_command"] is None
        else round(st["e2e_marginal_ms_per_added_command"], 2),
        "ms_per_added_command_ref_equiv": st["ref_equiv_ms_per_added_command"],
        "rollbacks_executed": rollbacks,
        "data": "synthetic multi-command transcripts + random-init weights (grammar-constrained decode)",
    }


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--config", type=int, nargs="+", default=[2, 3])
    ap.add_argument("--per-stream", type=int, default=4)
    ap.add_argument("--warmup", type=int, default=1)
    args = ap.parse_args()
    from loqa_hub_amd.messaging.nats_server import NATSServer
    from loqa_hub_amd.messaging.nats_service import NATSService
    dev = torch.device("cuda", 0)
    loop = asyncio.new_event_loop()
    asyncio.set_event_loop(loop)
    srv = loop.run_until_complete(NATSServer("127.0.0.1", 0).start())
    nats = NATSService(srv.url)
    loop.run_until_complete(nats.connect())
    for c in args.config:
        res = config_3(args, dev, nats) if c == 3 else config_2_or_5(c, args, dev, nats)
        print(json.dumps(res), flush=True)
        torch.cuda.empty_cache()
    loop.run_until_complete(nats.close())
    loop.run_until_complete(srv.stop())
    return 0


if __name__ == "__main__":
    sys.exit(main())
