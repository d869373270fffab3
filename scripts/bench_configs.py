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
  --config 5  Whisper-large-v3 + Llama-3-70B + progressive VITS speech of every
              reply. --tp 1: ONE GPU, compact single-copy weights (fused
              decode layout, chunked fused prefill: 70B bf16 = 141 GB fits in
              288 GB HBM3E). --tp N: the config's own layout, one process per
              GPU under torchrun (rank 0: hub pipeline + TP leader, ranks
              1..N-1: followers; parallel/tp_serving.py):
                torchrun --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
                  --master-port 29533 scripts/bench_configs.py --config 5 --tp 8
              --share-gpu N rehearses that layout with N ranks on cuda:0 (a
              1-GPU box: correct, not a timing of the xGMI links). 8 closed-loop
              streams, utterances/s, ms per added command, first-phrase audio
              latency (phrases are spoken while the decode runs) and the TTS
              share of the wall time.

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


def _progressive_loop(pipe, utts, streams: int, per_stream: int, tts):
    """Closed-loop clients whose replies are spoken progressively from the
    live decode (streaming/progressive.py) - the config-5 serving path."""
    from loqa_hub_amd.streaming.audio_pipeline import StreamingAudioPipeline
    from loqa_hub_amd.streaming.progressive import ProgressiveSpeech
    speech_pipe = StreamingAudioPipeline(tts)
    jobs, speech = [], []

    async def client(ci):
        for k in range(per_stream):
            u = utts[(ci * per_stream + k) % len(utts)]
            j = PipelineJob(u.relay_id, f"c{ci}-{k}", u.pcm, transcript_hint=u.text)
            sp = ProgressiveSpeech(u.relay_id, pipe.llm.tok, speech_pipe, None)
            j.on_tokens = sp.on_tokens
            j.t["start"] = sp.t_start = time.perf_counter()
            await pipe.submit(j)
            await sp.finish(j.multi.commands[0].response if j.multi and j.multi.commands else "")
            j.t["tts_done"] = time.perf_counter()
            jobs.append(j)
            speech.append(sp)

    async def main():
        t0 = time.perf_counter()
        await asyncio.gather(*[client(c) for c in range(streams)])
        return time.perf_counter() - t0
    wall = asyncio.get_event_loop().run_until_complete(main())
    return jobs, wall, speech


def _slope(xs, ys):
    """Least-squares slope of ys over xs (None with < 2 distinct xs)."""
    if len(set(xs)) < 2:
        return None
    return round(float(np.polyfit(np.asarray(xs, float), np.asarray(ys, float), 1)[0]), 3)


def config_2_or_5(cfg_id: int, args, dev, nats, tp_info=None) -> dict:
    if cfg_id == 2:
        stt_name, llm_name, streams = "whisper-base", "tinyllama", 1
    else:
        stt_name, llm_name, streams = "whisper-large-v3", "llama3-70b", 8
    if getattr(args, "streams", 0):
        streams = args.streams
    t0 = time.perf_counter()
    stt = STTEngine(whisper_config(stt_name), dev, seed=0, max_batch=8)
    tp = tp_info.world if tp_info is not None else 1
    if tp > 1:
        from loqa_hub_amd.parallel.tp_serving import build_tp_llm
        llm = build_tp_llm(llama_config(llm_name), tp_info, seed=0, max_seqs=8, max_seq_len=1024,
                           compact=args.compact)
    else:
        # 70B at TP=1: one weight copy in the fused decode layout (141 GB)
        llm = LLMEngine(llama_config(llm_name), dev, seed=0, max_seqs=8, max_seq_len=1024,
                        compact=llm_name == "llama3-70b")
    pipe = VoicePipeline(stt, llm, nats, min_response_tokens=8, max_batch=8)
    pipe.warmup()
    tts = None
    if cfg_id == 5 and not getattr(args, "no_tts", False):
        from loqa_hub_amd.engine.tts_engine import VitsTTSEngine
        tts = VitsTTSEngine(vits_config("vits-ljs"), dev, seed=0)
    init_s = time.perf_counter() - t0
    utts = make_batch(0, 16, [1, 2, 3, 4])
    speech = []
    if tts is not None:
        _progressive_loop(pipe, utts, streams, args.warmup, tts)          # warm-up
        s0, t0s = dict(llm.stats), dict(tts.stats)
        per_stream = args.per_stream
        jobs, wall, speech = _progressive_loop(pipe, utts, streams, per_stream, tts)
    else:
        _closed_loop(pipe, utts, streams, args.warmup)           # warm-up
        s0 = dict(llm.stats)
        per_stream = args.per_stream * (4 if streams == 1 else 1)
        jobs, wall, _ = _closed_loop(pipe, utts, streams, per_stream)
    st = added_command_stats(jobs)
    lat = _lat(jobs, "tts_done" if tts is not None else "queue_done")
    stt_ms = [(j.t["stt_done"] - j.t["start"]) * 1e3 for j in jobs]
    steps = llm.stats["decode_steps"] - s0["decode_steps"]
    out = {
        "config": cfg_id, "model": f"{stt_name} + {llm_name}" + (" + vits-ljs" if tts else ""),
        "n_gpus": tp, "tp": tp, "streams": streams, "utterances": len(jobs), "dtype": "bf16",
        "share_gpu": bool(args.share_gpu),
        "utterances_per_s": round(len(jobs) / wall, 3),
        "latency_ms_p50": round(float(np.median(lat)), 1),
        "latency_ms_p90": round(float(np.percentile(lat, 90)), 1),
        "stt_ms_mean": round(float(np.mean(stt_ms)), 1),
        "ms_per_added_command_e2e_marginal": None if st["e2e_marginal_ms_per_added_command"] is None
        else round(st["e2e_marginal_ms_per_added_command"], 2),
        "ms_per_added_command_ref_equiv": st["ref_equiv_ms_per_added_command"],
        "llm_ms_per_decode_step": round((llm.stats["decode_s"] - s0["decode_s"]) / max(1, steps) * 1e3, 3),
        # measured: the decode steps an utterance's parse sampled in, per added
        # command (slope over the command counts) - the step count a TP=8
        # projection multiplies its rank step by for a single stream
        "decode_steps_per_added_command": _slope([j.n_commands for j in jobs],
                                                 [j.llm_steps for j in jobs]),
        "stt_ms_per_added_command": _slope([j.n_commands for j in jobs], stt_ms),
        # the added command's cost in decode steps of this run (marginal ms /
        # ms per step): what a TP=8 projection multiplies its rank step by
        "steps_per_added_command": (None if not st["e2e_marginal_ms_per_added_command"] or not steps
                                    else round(st["e2e_marginal_ms_per_added_command"]
                                               / ((llm.stats["decode_s"] - s0["decode_s"]) / steps * 1e3), 2)),
        "command_count_match": float(np.mean([j.n_commands == j.n_expected for j in jobs])),
        "init_s": round(init_s, 1),
        "fused_gemm_tuning": {f"{k[0]}:{k[1]}x{k[2]}:M{k[3]}": list(v) for k, v in ops._FSPLITS.items()},
        "data": "synthetic speech-like PCM16 + random-init weights (teacher-forced STT)",
    }
    if speech:
        fa = [sp.t_first_audio - sp.t_start for sp in speech if sp.t_first_audio]
        before = [sp.t_first_audio < j.t["llm_done"] for sp, j in zip(speech, jobs)
                  if sp.t_first_audio and "llm_done" in j.t]
        tts_s = tts.stats.get("gpu_s", 0.0) - t0s.get("gpu_s", 0.0)
        out.update({
            "first_phrase_audio_ms_p50": round(float(np.median(fa)) * 1e3, 1) if fa else None,
            "first_phrase_audio_ms_p90": round(float(np.percentile(fa, 90)) * 1e3, 1) if fa else None,
            "first_audio_before_decode_done": round(float(np.mean(before)), 3) if before else None,
            "phrases_per_reply": round(float(np.mean([len(sp.chunks) for sp in speech])), 2),
            "tts_batches": tts.stats["batches"] - t0s["batches"],
            "tts_share_of_wall": round(tts_s / wall, 4),
        })
    if tp > 1:
        llm.stop()
        car = llm.tp.car
        out["tp_collective_calls"] = car.calls if car is not None else None
        out["tp_collective_error"] = bool(car.error()) if car is not None else None
    return out


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

    async def one(i, u, faults=True, out=None):
        nonlocal rollbacks
        j = PipelineJob(u.relay_id, f"t{i}", u.pcm, transcript_hint=u.text)
        j.t["start"] = time.perf_counter()
        j.transcription = to_transcription_result(u.text.split(" ", 2)[-1] if u.text.startswith("hey loqa")
                                                  else u.text)
        toks = []
        j.on_tokens = lambda ids: toks.append((time.perf_counter(), len(ids)))
        fault = faults and i % 4 == 3
        if faults:
            set_faults("nats_down%0.5" if fault else "")
        await pipe._llm_stage([j])
        if faults:
            set_faults("")
        if fault and j.queue is not None and j.queue.rollback_occurred:
            rollbacks += 1
        t_first = toks[1][0] if len(toks) > 1 else toks[0][0]
        n_tok = sum(n for _, n in toks)
        dur = toks[-1][0] - toks[0][0]
        (rows if out is None else out).append((j, (t_first - j.t["start"]) * 1e3, n_tok / max(dur, 1e-9)))

    loaded: list = []

    async def main():
        for i, u in enumerate(utts[:4]):
            await one(i, u)             # warm-up
        rows.clear()
        for k in range(args.per_stream * 4):
            await one(k, utts[k % len(utts)])
        if args.concurrency > 1:
            # the same streaming path under load: C closed-loop text streams
            # sharing the continuous batch (no fault injection: it is global)
            async def client(c):
                for k in range(args.per_stream):
                    await one(100 + c * args.per_stream + k, utts[(c + k) % len(utts)], faults=False,
                              out=loaded)
            t0 = time.perf_counter()
            await asyncio.gather(*[client(c) for c in range(args.concurrency)])
            loaded.append(time.perf_counter() - t0)
    loop.run_until_complete(main())
    jobs = [r[0] for r in rows]
    st = added_command_stats(jobs)
    llm.stop()
    extra = {}
    if loaded:
        wall = loaded.pop()
        lj = [r[0] for r in loaded]
        lst = added_command_stats(lj)
        extra = {
            "loaded_streams": args.concurrency,
            "loaded_utterances_per_s": round(len(lj) / wall, 2),
            "loaded_first_token_ms_p50": round(float(np.median([r[1] for r in loaded])), 2),
            "loaded_first_token_ms_p90": round(float(np.percentile([r[1] for r in loaded], 90)), 2),
            "loaded_stream_tokens_per_s_p50": round(float(np.median([r[2] for r in loaded])), 1),
            "loaded_ms_per_added_command_e2e_marginal":
                None if lst["e2e_marginal_ms_per_added_command"] is None
                else round(lst["e2e_marginal_ms_per_added_command"], 2),
        }
    return {
        "config": 3, "model": "llama3-8b", "n_gpus": 1, "tp": 1, "dtype": "bf16",
        "utterances": len(jobs),
        "first_token_ms_p50": round(float(np.median([r[1] for r in rows])), 2),
        "stream_tokens_per_s_p50": round(float(np.median([r[2] for r in rows])), 1),
        "ms_per_added_command_e2e_marginal": None if st["e2e_marginal_ms_per_added_command"] is None
        else round(st["e2e_marginal_ms_per_added_command"], 2),
        "ms_per_added_command_ref_equiv": st["ref_equiv_ms_per_added_command"],
        "rollbacks_executed": rollbacks,
        **extra,
        "data": "synthetic multi-command transcripts + random-init weights (grammar-constrained decode)",
    }


def _heartbeat(tag: str, every: float = 20.0) -> None:
    """Progress line every ``every`` seconds (long start-ups stay visibly alive)."""
    import threading
    t0 = time.perf_counter()

    def beat():
        while True:
            time.sleep(every)
            print(f"[{tag}] alive {time.perf_counter() - t0:.0f} s", file=sys.stderr, flush=True)
    threading.Thread(target=beat, daemon=True).start()


def _tp_rank_main(args) -> int:
    """Rank body of ``--config 5 --tp N`` (torchrun or --share-gpu)."""
    from loqa_hub_amd.parallel.tp_serving import init_tp, run_follower
    info = init_tp(args.tp)
    if info.rank == 0:
        _heartbeat("tp leader")
    if args.share_gpu:
        info.device = torch.device("cuda", 0)
        torch.cuda.set_device(0)
    if info.rank != 0:
        from loqa_hub_amd.parallel.tp_serving import build_tp_llm
        eng = build_tp_llm(llama_config("llama3-70b"), info, seed=0, max_seqs=8, max_seq_len=1024,
                           compact=args.compact)
        run_follower(eng)
        return 0
    from loqa_hub_amd.messaging.nats_server import NATSServer
    from loqa_hub_amd.messaging.nats_service import NATSService
    loop = asyncio.new_event_loop()
    asyncio.set_event_loop(loop)
    srv = loop.run_until_complete(NATSServer("127.0.0.1", 0).start())
    nats = NATSService(srv.url)
    loop.run_until_complete(nats.connect())
    res = config_2_or_5(5, args, info.device, nats, tp_info=info)
    print(json.dumps(res), flush=True)
    loop.run_until_complete(nats.close())
    loop.run_until_complete(srv.stop())
    return 0


def _share_gpu_worker(rank, world, port, argv):
    os.environ.update(RANK=str(rank), LOCAL_RANK="0", WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      LOQA_NO_TUNE="1")   # ranks sharing one GPU cannot time anything
    # N processes x HIP's default 4 hardware queues oversubscribe the GPU's
    # queue slots and the scheduler time-slices the ranks (~28x slower steps,
    # profiles/r3_tp8_share_hwq.txt): one queue per follower, two for the
    # leader (decoders, prefill, STT, TTS streams)
    os.environ["GPU_MAX_HW_QUEUES"] = "2" if rank == 0 else "1"
    sys.argv = [sys.argv[0]] + argv
    main()


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--config", type=int, nargs="+", default=[2, 3])
    ap.add_argument("--per-stream", type=int, default=4)
    ap.add_argument("--streams", type=int, default=0,
                    help="configs 2 / 5: closed-loop streams (0: the config's own, 1 / 8)")
    ap.add_argument("--no-tts", action="store_true",
                    help="config 5: no progressive VITS (the LLM's steps per added command alone)")
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--tp", type=int, default=1, help="config 5: tensor-parallel degree")
    ap.add_argument("--concurrency", type=int, default=8,
                    help="config 3: closed-loop text streams of the loaded run (1: unloaded only)")
    ap.add_argument("--share-gpu", action="store_true",
                    help="TP ranks share cuda:0 (spawned here when not under torchrun)")
    ap.add_argument("--compact", action="store_true",
                    help="TP: single-copy fused weights (needed when ranks share a GPU)")
    args = ap.parse_args()
    if args.tp > 1:
        if args.config != [5]:
            ap.error("--tp applies to --config 5 only")
        if args.share_gpu and "WORLD_SIZE" not in os.environ:
            # spawn the ranks before this process touches the GPU
            import socket

            import torch.multiprocessing as mp
            with socket.socket() as sk:
                sk.bind(("127.0.0.1", 0))
                port = sk.getsockname()[1]
            os.environ["LOQA_NO_TUNE"] = "1"     # inherited by the spawned ranks
            mp.start_processes(_share_gpu_worker, args=(args.tp, port, sys.argv[1:]),
                               nprocs=args.tp, join=True, start_method="spawn")
            return 0
        return _tp_rank_main(args)
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
