#!/usr/bin/env python3
"""Headline benchmark: multi-command utterances through the on-GPU voice pipeline.

BASELINE.json metric: "ms per added command (multi-cmd utterance) + utterances/sec
at 1/2/4/8 MI355X"; config 4: 64 concurrent audio streams, Whisper-large-v3 +
Llama-3-8B intent, DP=8 (8 streams per GPU -> weak scaling: per-GPU work fixed).

One step = every rank processes B utterances end to end (--mode batch: the
rank-0 router scatters the step's PCM16 over RCCL; the hub / closed modes
draw each rank's utterances locally from the shared seed) -> fused PCM convert/RMS ->
  log-mel -> Whisper-large-v3 encoder + teacher-forced greedy decode ->
  wake-word strip -> ONE grammar-constrained Llama-3-8B multi-command decode
  (verbatim reference prompt, jump-forward JSON) -> command queue with rollback
  -> NATS publishes (embedded broker) -> per-utterance records all_gathered.

Prints ONE JSON line (rank 0). ``value`` = utterances/s over all GPUs;
ms-per-added-command (both BASELINE.md definitions) is reported alongside.
Random-init weights, synthetic speech-like audio (no network / checkpoints).

Modes: ``hub`` (default, the headline - BASELINE config 4 is "64 concurrent
gRPC audio streams"): the SERVED path, the reference's hot path
(``audio_service.go:926-1043``) - a ``HubServer`` per GPU (per rank under
torchrun) with B simulated relays, each a closed loop of gRPC ``StreamAudio``
calls (wake-word chunk, 100 ms PCM16 chunks, end of speech), per-relay-group
arbitration with the single-relay bypass (every bench relay is alone in its
group; ``--no-bypass`` waits out the window), the GPU voice processor,
voice-event writes to SQLite and the command queue on NATS. After the timed
steps, ``--window-steps`` more run with the reference's 300 ms window
(``window_300ms``, a secondary field). ``closed``: B closed-loop streams per
GPU submit straight into the voice pipeline (no gRPC). ``batch``: lockstep
batches of B.

``--gpus N`` must match the launch: under torchrun WORLD_SIZE must equal N
(else exit 2); without torchrun and N > 1 the bench launches
``torch.distributed.run`` itself (before touching the GPU) and exits with its
status.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import sys
import threading
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from loqa_hub_amd import ops  # noqa: E402
from loqa_hub_amd.engine.llm_engine import LLMEngine  # noqa: E402
from loqa_hub_amd.engine.pipeline import PipelineJob, VoicePipeline, added_command_stats  # noqa: E402
from loqa_hub_amd.engine.stt_engine import STTEngine  # noqa: E402
from loqa_hub_amd.engine.synthetic import make_batch, make_unique  # noqa: E402
from loqa_hub_amd.messaging.nats_server import NATSServer  # noqa: E402
from loqa_hub_amd.messaging.nats_service import NATSService  # noqa: E402
from loqa_hub_amd.models.configs import llama_config, whisper_config  # noqa: E402
from loqa_hub_amd.parallel import dist as pdist  # noqa: E402
from loqa_hub_amd.parallel.dp_router import gather_records, scatter_pcm, slot_len_for  # noqa: E402

BASELINE_MS_PER_ADDED_COMMAND = 200.0


def spawn_broker() -> tuple[int, "subprocess.Popen"]:
    """NATS broker in its own process (as nats-server is in a deployment): the
    serving process's GIL carries no broker work, which matters most on rank 0
    of a DP run, where every rank publishes. Started before anything touches
    the GPU; it exits when our end of its stdin closes."""
    import subprocess
    p = subprocess.Popen([sys.executable, "-m", "loqa_hub_amd.messaging.nats_server"],
                         stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True,
                         cwd=os.path.dirname(os.path.abspath(__file__)))
    line = p.stdout.readline().split()
    if len(line) != 2 or line[0] != "port":
        p.kill()
        raise RuntimeError(f"NATS broker did not start: {line}")
    return int(line[1]), p


def start_broker() -> tuple[int, threading.Thread]:
    ready = threading.Event()
    box = {}

    def run():
        loop = asyncio.new_event_loop()
        srv = loop.run_until_complete(NATSServer("127.0.0.1", 0).start())
        box["port"] = srv.port
        ready.set()
        loop.run_forever()

    t = threading.Thread(target=run, daemon=True)
    t.start()
    ready.wait(10)
    return box["port"], t


async def _start_hub(args, pipe, nats_port: int, info, texts: dict):
    """The served hub of --mode hub on this rank's GPU pipeline. ``texts``:
    relay -> its utterances' transcripts in sending order (the teacher-forcing
    hints of the random-init Whisper; each processed utterance takes the next)."""
    import collections
    import tempfile

    from loqa_hub_amd import config as cfgmod
    from loqa_hub_amd.server import HubServer, build_bridge
    from loqa_hub_amd.transport.voice_processor import GPUVoiceProcessor
    db = os.path.join(tempfile.mkdtemp(prefix="loqa-bench-"), "hub.db")
    cfg = cfgmod.load({"LOQA_DB_PATH": db, "NATS_URL": f"nats://127.0.0.1:{nats_port}",
                       "ARBITRATION_SCOPE": "per_relay_group",
                       "ARBITRATION_WINDOW_DURATION": f"{args.window_ms}ms",
                       "ARBITRATION_SINGLE_RELAY_BYPASS": "true" if args.bypass else "false"})
    fifo = {r: collections.deque(t) for r, t in texts.items()}

    def hint(relay: str):
        q = fifo.get(relay)
        return q.popleft() if q else None
    srv = HubServer(cfg, skills_dir=os.path.join(os.path.dirname(db), "skills"),
                    skills_config_store=os.path.join(os.path.dirname(db), "skillcfg"),
                    transcript_hints=hint)
    await srv._connect_nats()
    srv.processor = GPUVoiceProcessor(pipe, max_batch=pipe.max_batch,
                                      bridge=None if os.environ.get("LOQA_BENCH_NO_BRIDGE") == "1"
                                      else build_bridge(srv.skills), batch_window=0.002)
    await srv.start(host="127.0.0.1", http_port=0, grpc_port=0)
    return srv


class CommandCounter:
    """--mode hub: the commands each served utterance actually published on
    ``loqa.voice.commands`` (counted per request id), matched to the relay's
    utterances through the voice events (one per processed utterance, in
    order per relay) - the parsed command count, not the expected one."""

    def __init__(self, client):
        self.client = client
        self.per_request: dict[str, int] = {}

    @classmethod
    async def start(cls, url: str) -> "CommandCounter":
        from loqa_hub_amd.messaging.nats_client import NATSClient
        c = NATSClient(name="bench-command-counter")
        await c.connect(url)
        self = cls(c)

        def on_msg(m):
            rid = json.loads(m.data).get("request_id", "")
            self.per_request[rid] = self.per_request.get(rid, 0) + 1
        await c.subscribe("loqa.voice.commands", on_msg)
        await c.flush()
        return self

    async def records(self, srv, hub_recs: dict) -> list[list[float]]:
        """[parsed commands, expected, ok, latency ms] per timed utterance."""
        from loqa_hub_amd.storage.voice_events_store import ListOptions
        await asyncio.sleep(0.2)
        await self.client.flush()
        evs = srv.events.list(ListOptions(sort_by="timestamp", sort_order="ASC"))
        by_relay: dict[str, list[str]] = {}
        for ev in evs:
            by_relay.setdefault(ev.relay_id, []).append(ev.request_id)
        out = []
        for relay, recs in hub_recs.items():
            rids = by_relay.get(relay, [])[-len(recs):]
            rids = [""] * (len(recs) - len(rids)) + rids
            for (expected, ok, lat), rid in zip(recs, rids):
                out.append([float(self.per_request.get(rid, 0)), float(expected), ok, lat])
        return out

    async def close(self) -> None:
        await self.client.close()


def hub_summary(srv, recs: list, args, events_before: int = 0) -> tuple[float | None, dict]:
    """Served-path statistics: the end-to-end marginal cost of an added command
    (slope of the relay-side latency over the parsed command count) and the
    hub's own counters. ``voice_events``: events stored during the timed steps
    (``events_before`` = the count when they started: warm-up utterances are
    stored too), one per timed utterance; ``voice_events_total`` all of them."""
    from loqa_hub_amd.storage.voice_events_store import ListOptions
    r = np.array(recs, dtype=np.float64).reshape(-1, 4)
    slope = (float(np.polyfit(r[:, 0], r[:, 3], 1)[0])
             if len(r) and len(set(r[:, 0])) >= 2 else None)
    st = srv.processor.stats
    gap = (round(1e3 * st["eos_enc_gap_s"] / st["eos_enc_n"], 3)
           if st.get("eos_enc_n") else None)
    total = srv.events.count(ListOptions())
    return slope, {"voice_events": total - events_before, "voice_events_total": total,
                   "timed_utterances": len(r),
                   "end_of_speech_to_encoder_ms": gap,
                   "encode_span_ms": (round(1e3 * st["enc_span_s"] / st["eos_enc_n"], 3)
                                      if st.get("eos_enc_n") and "enc_span_s" in st else None),
                   "paced": bool(getattr(args, "paced", False)),
                   "audio_service": dict(srv.audio_service.stats),
                   "processor": dict(srv.processor.stats),
                   "latency_ms_p50": round(float(np.median(r[:, 3])), 1) if len(r) else None,
                   "latency_ms_p90": round(float(np.percentile(r[:, 3], 90)), 1) if len(r) else None,
                   "window_ms": args.window_ms}


def run_hub_dp(args) -> int:
    """``--mode hub`` over ``--gpus N`` (or with ``--tts``): the served hub as
    deployed for BASELINE config 4 - one front-end process (gRPC relays,
    per-group arbitration, voice events in SQLite) and one worker process per
    GPU, each with the full composition (``server.build_dp_processor``). B
    relays per GPU, each a closed loop of StreamAudio calls. The front end
    never touches a GPU. ``LOQA_DIST_SHARE_GPU=1``: every worker on cuda:0
    (the rehearsal on a one-GPU box)."""
    import tempfile

    import grpc

    from loqa_hub_amd import config as cfgmod
    from loqa_hub_amd.server import HubServer, build_dp_processor
    from loqa_hub_amd.transport.audio_proto import AudioChunk, stream_audio_stub
    N, B = args.gpus, args.batch_per_gpu
    mix = [int(x) for x in args.mix.split(",")]
    if args.cpu_smoke:
        args.stt, args.llm, args.tts_model = "test-whisper", "test-tiny", "test-vits"
    port, broker = spawn_broker()
    tmp = tempfile.mkdtemp(prefix="loqa-bench-hub-")
    cfg = cfgmod.load({"LOQA_DB_PATH": os.path.join(tmp, "hub.db"),
                       "NATS_URL": f"nats://127.0.0.1:{port}",
                       "ARBITRATION_SCOPE": "per_relay_group",
                       "ARBITRATION_WINDOW_DURATION": f"{args.window_ms}ms",
                       "ARBITRATION_SINGLE_RELAY_BYPASS": "true" if args.bypass else "false",
                       "HUB_STT_MODEL": args.stt, "HUB_LLM_MODEL": args.llm,
                       "HUB_TTS_MODEL": args.tts_model, "HUB_MAX_BATCH": str(max(B, 8)),
                       "HUB_TTS_BACKEND": "gpu" if args.tts else "none",
                       "STREAMING_ENABLED": "true" if args.tts else "false",
                       "HUB_USE_GRAPHS": "false" if args.no_graphs else "true",
                       "HUB_SEED": str(args.seed)})
    device = ("cpu" if args.cpu_smoke else
              "cuda:0" if os.environ.get("LOQA_DIST_SHARE_GPU", "0") == "1" else "cuda")
    n_per_stream = args.warmup + args.steps
    from loqa_hub_amd.engine.synthetic import make_unique
    counts = [mix[(ci + k) % len(mix)] for ci in range(N * B) for k in range(n_per_stream)]
    uniq = make_unique(args.seed, counts)
    hints: dict[str, str] = {}
    hub_recs: dict[str, list] = {}

    async def main() -> dict:
        srv = HubServer(cfg, skills_dir=os.path.join(tmp, "skills"),
                        skills_config_store=os.path.join(tmp, "skillcfg"),
                        transcript_hints=hints.get)
        await srv._connect_nats()
        t_init = time.perf_counter()
        srv.processor = await build_dp_processor(cfg, N, srv.nats.url, device=device,
                                                 skills_dir=os.path.join(tmp, "skills"),
                                                 skills_config_store=os.path.join(tmp, "skillcfg"))
        t_init = time.perf_counter() - t_init
        await srv.start(host="127.0.0.1", http_port=0, grpc_port=0)
        counter = await CommandCounter.start(srv.nats.url)

        async def client(ci: int, ch, n: int, record: bool) -> None:
            call = stream_audio_stub(ch)
            relay = f"relay-{ci}"
            for k in range(n):
                u = uniq[ci * n_per_stream + k + (args.warmup if record else 0)]
                hints[relay] = u.text
                data = np.ascontiguousarray(u.pcm, dtype="<i2").tobytes()
                wake, rest = data[:9600], data[9600:]

                async def chunks():
                    yield AudioChunk(relay_id=relay, audio_data=wake, sample_rate=16000,
                                     is_wake_word=True)
                    for o in range(0, max(len(rest), 1), 3200):
                        yield AudioChunk(relay_id=relay, audio_data=rest[o:o + 3200],
                                         sample_rate=16000, is_end_of_speech=o + 3200 >= len(rest))
                t_s = time.perf_counter()
                got = [r async for r in call(chunks())]
                lat = (time.perf_counter() - t_s) * 1e3
                if record:
                    hub_recs.setdefault(relay, []).append(
                        [u.n_commands, float(bool(got) and got[-1].success), lat])

        async def run(n: int, record: bool) -> None:
            async with grpc.aio.insecure_channel(f"127.0.0.1:{srv.grpc_port}") as ch:
                await asyncio.gather(*[client(ci, ch, n, record) for ci in range(N * B)])
        try:
            from loqa_hub_amd.storage.voice_events_store import ListOptions
            await run(args.warmup, False)
            ev0 = srv.events.count(ListOptions())
            t0 = time.perf_counter()
            await run(args.steps, True)
            elapsed = time.perf_counter() - t0
            recs = await counter.records(srv, hub_recs)
            slope, hub_stats = hub_summary(srv, recs, args, ev0)
            hub_stats["dp"] = srv.processor.metrics()
            ps = srv.processor.stats
            if args.tts and ps.get("tts_phrases"):
                sr = 22050.0
                hub_stats["tts"] = {
                    "phrases_per_s": round(ps["tts_phrases"] / max(elapsed, 1e-9), 2),
                    "audio_s_per_wall_s": round(ps["tts_samples"] / sr / max(elapsed, 1e-9), 2),
                    "gpu_s_per_audio_s": round(ps["tts_gpu_s"] / max(ps["tts_samples"] / sr, 1e-9), 4),
                    "host_launch_ms_per_batch": round(1e3 * ps.get("tts_launch_s", 0.0)
                                                      / max(ps.get("tts_batches", 1), 1), 3),
                    "phrases_per_batch": round(ps["tts_phrases"] / max(ps.get("tts_batches", 1), 1), 2),
                    "note": "counters since start (warm-up included)"}
            if srv.streaming is not None:
                hub_stats["streaming"] = srv.streaming.metrics.get_aggregate_metrics().to_json()
        finally:
            await counter.close()
            await srv.stop()
        r = np.array(recs, dtype=np.float64).reshape(-1, 4)
        return {"elapsed": elapsed, "slope": slope, "hub": hub_stats, "init_s": t_init,
                "ok": float(r[:, 2].mean()) if len(r) else 0.0,
                "match": float((r[:, 0] == r[:, 1]).mean()) if len(r) else 0.0}
    try:
        res = asyncio.run(main())
    finally:
        broker.stdin.close()
        broker.wait(timeout=10)
    value = N * B * args.steps / res["elapsed"]
    e2e = res["slope"]
    print(json.dumps({
        "metric": ("utterances_per_sec (multi-command utterances; ms per added command "
                   "reported alongside)"),
        "value": round(value, 3), "unit": "utterances/s", "n_gpus": N, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(res["elapsed"] / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
        "data": ("synthetic speech-like PCM16 over gRPC relays, every utterance a distinct "
                 "transcript + random-init weights (teacher-forced STT, grammar-constrained LLM)"),
        "config": {"model": f"{args.stt} + {args.llm}" + (
            f" + {args.tts_model}" if args.tts and not os.environ.get("HUB_TTS_CHECKPOINT") else
            f" + VITS checkpoint {os.path.basename(os.path.normpath(os.environ['HUB_TTS_CHECKPOINT']))}"
            if args.tts else ""),
                   "global_batch": N * B, "seq_len": 1500, "parallelism": f"dp{N}",
                   "commands_mix": mix, "baseline_config": 4, "mode": "hub",
                   "served": "front end + one worker process per GPU",
                   "shared_gpu": device == "cuda:0", "concurrent_streams_per_gpu": B,
                   "tts": args.tts},
        "ms_per_added_command_e2e_marginal": None if e2e is None else round(e2e, 3),
        "baseline_ms_per_added_command": BASELINE_MS_PER_ADDED_COMMAND,
        "added_command_speedup_vs_baseline": (None if not e2e or e2e <= 0 else
                                              round(BASELINE_MS_PER_ADDED_COMMAND / e2e, 3)),
        "queue_success_rate": round(res["ok"], 4),
        "command_count_match_rate": round(res["match"], 4),
        "hub": res["hub"], "init_s": round(res["init_s"], 2)}), flush=True)
    return 0


def relaunch(n: int, argv: list[str]) -> int:
    """``--gpus N`` without torchrun: run this bench under torch.distributed.run
    with N ranks (a child process; nothing here has touched the GPU)."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__),
           *argv]
    return subprocess.call(cmd)


def rank_device_problem(args) -> str | None:
    """Fail-fast check before any collective: every rank of a GPU run needs a
    GPU of its own (LOCAL_RANK < visible devices; device_count() does not
    initialise the GPU). None when the launch is sound."""
    if args.cpu_smoke:
        return None
    n_dev = torch.cuda.device_count()
    local = int(os.environ.get("LOCAL_RANK", "0"))
    share = os.environ.get("LOQA_DIST_SHARE_GPU", "0") == "1"
    if n_dev == 0:
        return "no GPU visible (HIP_VISIBLE_DEVICES?) and --cpu-smoke not given"
    if not share and local >= n_dev:
        return (f"rank {os.environ.get('RANK', '0')} (LOCAL_RANK {local}) has no GPU: "
                f"{n_dev} visible for --gpus {args.gpus} (one rank per GPU)")
    return None


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (default: WORLD_SIZE under torchrun, else 1)")
    # 8 utterances per stream: a whole number of passes over the 4-way command
    # mix for every stream (5 ends on an unbalanced tail: measured 17.4-17.5
    # vs 18.7-18.9 utt/s at 4, 8 and 12)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch-per-gpu", type=int, default=8)
    ap.add_argument("--stt", default="whisper-large-v3")
    ap.add_argument("--llm", default="llama3-8b")
    ap.add_argument("--mix", default="1,2,3,4", help="commands per utterance, cycled")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--mode", choices=["closed", "hub", "batch"], default="hub",
                    help="hub (default): B simulated relays per GPU over gRPC into the served "
                         "hub; closed: B concurrent closed-loop streams per GPU straight into "
                         "the pipeline (continuous batching); batch: lockstep batches of B")
    ap.add_argument("--paced", action="store_true",
                    help="--mode hub: relays send their speech in real time (100 ms chunks "
                         "every 100 ms); latency is then counted from the end of speech")
    ap.add_argument("--bypass", dest="bypass", action="store_true", default=True,
                    help="--mode hub (default on): a relay alone in its group wins at once "
                         "(ARBITRATION_SINGLE_RELAY_BYPASS; every bench relay is its own group)")
    ap.add_argument("--no-bypass", dest="bypass", action="store_false",
                    help="--mode hub: every relay waits out the arbitration window")
    ap.add_argument("--window-ms", type=float, default=300.0,
                    help="--mode hub: arbitration window (the reference's 300 ms)")
    ap.add_argument("--window-steps", type=int, default=4,
                    help="--mode hub with bypass: utterances per relay timed afterwards with the "
                         "bypass off (the window_300ms secondary field; 0: skip)")
    ap.add_argument("--inflight", type=int, default=2,
                    help="--mode batch: batches in flight (2: next batch's STT overlaps the decode)")
    ap.add_argument("--cpu-smoke", action="store_true", help="tiny models on CPU (plumbing test)")
    ap.add_argument("--stt-priority", type=int, default=-1,
                    help="HIP stream priority of the STT worker (-1 high, 0 normal)")
    ap.add_argument("--tts", action="store_true",
                    help="--mode hub: every reply spoken by on-GPU VITS (progressive)")
    ap.add_argument("--tts-model", default="vits-ljs")
    ap.add_argument("--served-dp", action="store_true",
                    help="--mode hub: serve through the DP front end + worker processes at any N")
    args = ap.parse_args(argv)

    world_env = os.environ.get("WORLD_SIZE")
    if args.gpus is None:
        args.gpus = int(world_env or "1")
    if args.mode == "hub" and world_env is None and (args.gpus > 1 or args.tts or args.served_dp):
        # the served multi-GPU hub: ONE front-end process (gRPC, arbitration,
        # events) over one worker process per GPU (parallel/dp_serving.py)
        return run_hub_dp(args)
    if world_env is None and args.gpus > 1:
        return relaunch(args.gpus, sys.argv[1:] if argv is None else list(argv))
    if int(world_env or "1") != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world_env}: launch one rank per "
              f"GPU (torchrun --nproc-per-node {args.gpus})", file=sys.stderr)
        return 2
    bad = rank_device_problem(args)
    if bad:
        print(f"bench.py: {bad}", file=sys.stderr)
        return 2
    if args.cpu_smoke:
        args.stt, args.llm = "test-whisper", "test-tiny"
    # event bus: one NATS broker for the node (rank 0 starts it), every rank
    # connects; a separate process unless LOQA_BENCH_BROKER=thread
    broker = None
    port = 0
    if int(os.environ.get("RANK", "0")) == 0:
        if os.environ.get("LOQA_BENCH_BROKER", "process") == "process":
            port, broker = spawn_broker()
        else:
            port = start_broker()[0]
    info = pdist.init_distributed(prefer_gpu=not args.cpu_smoke)
    dev = info.device

    if dev.type == "cuda":
        torch.backends.cuda.matmul.allow_tf32 = False

    if info.world > 1:
        # through the rendezvous store: the first RCCL collective waits until
        # the pipeline's own streams are in use (parallel/dist.py)
        port = int(pdist.store_exchange(info, "loqa_nats_port", str(port)))
    loop = asyncio.new_event_loop()
    nats = NATSService(f"nats://127.0.0.1:{port}")
    loop.run_until_complete(nats.connect())

    B = args.batch_per_gpu
    mix = [int(x) for x in args.mix.split(",")]
    t_init = time.perf_counter()
    stt = STTEngine(whisper_config(args.stt), dev, seed=args.seed, max_batch=max(B, 8))
    llm = LLMEngine(llama_config(args.llm), dev, seed=args.seed, max_seqs=max(B, 8), max_seq_len=1024,
                    use_graphs=not args.no_graphs)
    pipe = VoicePipeline(stt, llm, nats, min_response_tokens=8, max_batch=B,
                         stt_priority=args.stt_priority)
    pipe.warmup()
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    t_init = time.perf_counter() - t_init

    utts = make_batch(args.seed, info.world * B, mix)
    mine = utts[info.rank * B:(info.rank + 1) * B]
    per_rank = [[u.pcm for u in utts[r * B:(r + 1) * B]] for r in range(info.world)]
    slot = slot_len_for(per_rank)
    all_jobs: list[PipelineJob] = []

    async def step(record: bool, prev: asyncio.Future | None) -> None:
        dpcm = scatter_pcm(info, per_rank if info.rank == 0 else None, slot)
        jobs = [PipelineJob(u.relay_id, f"req-{info.rank}-{i}", u.pcm, transcript_hint=u.text)
                for i, u in enumerate(mine)]
        await pipe.process(jobs, device_pcm=dpcm)
        if prev is not None:
            await prev  # collectives stay in step order on every rank
        rec = torch.tensor([[j.n_commands, j.n_expected, float(j.queue is not None and j.queue.success),
                             (j.t.get("queue_done", j.t["start"]) - j.t["start"]) * 1e3]
                            for j in jobs], dtype=torch.float64)
        gathered = gather_records(info, rec)
        if record:
            all_jobs.extend(jobs)
            step.records.append(gathered.cpu())

    step.records = []

    async def run_batches(n: int, record: bool) -> None:
        """--mode batch: n lockstep batches of B utterances, up to
        ``--inflight`` batches in flight."""
        sem = asyncio.Semaphore(max(1, args.inflight))
        tasks: list[asyncio.Future] = []
        for _ in range(n):
            await sem.acquire()
            t = asyncio.ensure_future(step(record, tasks[-1] if tasks else None))
            t.add_done_callback(lambda _t: sem.release())
            tasks.append(t)
        await asyncio.gather(*tasks)

    # closed mode: every submission is a DISTINCT utterance (distinct
    # transcript -> distinct prompt, so only the template text before the
    # transcript can hit the prefix cache), drawn up front for the warmup and
    # timed rounds; each stream's command count cycles through the mix
    win_steps = args.window_steps if (args.mode == "hub" and args.bypass) else 0
    n_per_stream = args.warmup + args.steps + win_steps
    uniq = []
    if args.mode in ("closed", "hub"):
        counts = [mix[(ci + k) % len(mix)] for ci in range(B) for k in range(n_per_stream)]
        uniq = make_unique(args.seed, counts, offset=info.rank * B * n_per_stream)

    def next_utt(ci: int, k: int, record: bool, base: int | None = None):
        return uniq[ci * n_per_stream + k + (base if base is not None else
                                             args.warmup if record else 0)]

    async def run_closed(n: int, record: bool) -> None:
        """--mode closed: B concurrent relay streams per GPU, each a
        closed loop (its next utterance is sent when the previous one's reply
        is back); n utterances per stream. Arrivals are micro-batched for STT
        and join the running LLM decode batch (continuous batching)."""
        async def client(ci: int) -> None:
            for k in range(n):
                u = next_utt(ci, k, record)
                j = PipelineJob(u.relay_id, f"req-{info.rank}-{ci}-{k}", u.pcm,
                                transcript_hint=u.text)
                await pipe.submit(j)
                if record:
                    all_jobs.append(j)
                    recs_local.append([j.n_commands, j.n_expected,
                                       float(j.queue is not None and j.queue.success),
                                       (j.t.get("queue_done", j.t["start"]) - j.t["start"]) * 1e3])
        await asyncio.gather(*[client(ci) for ci in range(B)])

    recs_local: list[list[float]] = []
    hub_recs: dict[str, list] = {}

    hub = relays = None
    if args.mode == "hub":
        # the relays are devices of their own: a separate process drives them
        # over gRPC (transport/relay_sim.py), so their client work shares no
        # GIL with this hub's scheduler threads
        from loqa_hub_amd.transport.relay_sim import RelayProcess, relay_name, relay_utterances
        ru = relay_utterances(args.seed, mix, B, n_per_stream, info.rank)
        texts = {relay_name(info.rank, ci): [u.text for u in ru[ci]] for ci in range(B)}
        hub = loop.run_until_complete(_start_hub(args, pipe, port, info, texts))
        relays = RelayProcess(port=hub.grpc_port, nats_url=f"nats://127.0.0.1:{port}",
                              rank=info.rank, relays=B, seed=args.seed, mix=args.mix,
                              per_relay=n_per_stream, paced=args.paced,
                              cwd=os.path.dirname(os.path.abspath(__file__)))

    async def run_hub(n: int, record: bool, base: int | None = None) -> None:
        """--mode hub: B relays per GPU, each a closed loop of gRPC StreamAudio
        calls (wake-word chunk, 100 ms speech chunks, end of speech) into the
        served hub, driven by the relay simulator process; latency = first
        chunk sent -> response received (relay side). ``base``: index of the
        first utterance of each relay's list (distinct utterances)."""
        b0 = base if base is not None else (args.warmup if record else 0)
        out = await relays.run(b0, n)
        if record:
            for relay, expected, ok, lat, rid in out:
                hub_recs.setdefault(relay, []).append([expected, ok, lat, rid])

    def run(n: int, record: bool):
        if args.mode == "hub":
            return run_hub(n, record)
        return run_closed(n, record) if args.mode == "closed" else run_batches(n, record)

    loop.run_until_complete(run(args.warmup, False))
    pdist.barrier(info)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    s0 = dict(llm.stats)
    ev0 = 0
    if hub is not None:
        from loqa_hub_amd.storage.voice_events_store import ListOptions
        ev0 = hub.events.count(ListOptions())     # warm-up utterances' events
        hub.processor.job_sink = all_jobs         # per-phase timestamps of the timed utterances
    t0 = time.perf_counter()
    loop.run_until_complete(run(args.steps, True))
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    pdist.barrier(info)
    elapsed = pdist.max_over_ranks(info, time.perf_counter() - t0)
    if hub is not None:
        hub.processor.job_sink = None

    if hub is not None:
        # commands each timed utterance actually published on loqa.voice.commands
        # (observed by the relay process over NATS, keyed by the response's
        # request id) - the parsed command count, not the expected one
        # (the gRPC response carries no request id, as the reference's
        # sendSuccessResponse sets none: utterances are matched to the voice
        # events, one per processed utterance, in order per relay)
        per_req = loop.run_until_complete(relays.counts())
        from loqa_hub_amd.storage.voice_events_store import ListOptions
        evs = hub.events.list(ListOptions(sort_by="timestamp", sort_order="ASC"))
        by_relay: dict[str, list[str]] = {}
        for ev in evs:
            by_relay.setdefault(ev.relay_id, []).append(ev.request_id)
        recs_local = []
        for relay, recs in hub_recs.items():
            rids = by_relay.get(relay, [])[-len(recs):]
            rids = [""] * (len(recs) - len(rids)) + rids
            for (exp, ok, lat, _), rid in zip(recs, rids):
                recs_local.append([float(per_req.get(rid, 0)), float(exp), ok, lat])
    if args.mode in ("closed", "hub") and recs_local:
        step.records.append(gather_records(info, torch.tensor(recs_local, dtype=torch.float64)).cpu())
    stats = added_command_stats(all_jobs)
    hub_stats = None
    if hub is not None:
        stats["e2e_marginal_ms_per_added_command"], hub_stats = hub_summary(hub, recs_local, args, ev0)
    def _mean_ms(a, b):
        v = [j.t[b] - j.t[a] for j in all_jobs if a in j.t and b in j.t]
        return round(float(np.mean(v)) * 1e3, 2) if v else None
    phase_ms = {
        "stt": _mean_ms("start", "stt_done"),
        "stt_wait_encoder": _mean_ms("start", "enc0"),
        "stt_encode": _mean_ms("enc0", "enc1"),
        "stt_wait_decoder": _mean_ms("enc1", "dec0"),
        "stt_decode": _mean_ms("dec0", "stt_done"),
        "llm_total": _mean_ms("stt_done", "queue_done"),
        "llm_prefill": round((llm.stats["prefill_s"] - s0["prefill_s"]) / args.steps * 1e3, 2),
        "llm_decode": round((llm.stats["decode_s"] - s0["decode_s"]) / args.steps * 1e3, 2),
        "llm_decode_steps": (llm.stats["decode_steps"] - s0["decode_steps"]) / args.steps,
        # chunked prompt passes (LOQA_CHUNK_PREFILL): passes that carry prompt
        # chunks together with the live sequences' next feeds
        "llm_mixed": round((llm.stats.get("mixed_s", 0.0) - s0.get("mixed_s", 0.0))
                           / args.steps * 1e3, 2),
        "llm_mixed_steps": (llm.stats.get("mixed_steps", 0) - s0.get("mixed_steps", 0)) / args.steps,
    }
    # counters as of the end of the timed steps (the window pass below runs more)
    llm_stats_t, stt_stats_t = dict(llm.stats), dict(stt.stats)
    window = None
    if hub is not None and win_steps > 0:
        # secondary: the same served path with every relay waiting out the
        # reference's arbitration window (audio_service.go:408-502)
        svc = hub.audio_service
        svc.single_relay_bypass = False
        pdist.barrier(info)
        tw = time.perf_counter()
        loop.run_until_complete(run_hub(win_steps, False, args.warmup + args.steps))
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        pdist.barrier(info)
        tw = pdist.max_over_ranks(info, time.perf_counter() - tw)
        window = {"window_ms": args.window_ms, "utterances_per_sec": round(info.world * B * win_steps / tw, 3),
                  "utterances": info.world * B * win_steps,
                  "note": "after the timed steps, single-relay bypass off: every utterance waits "
                          "out the arbitration window before STT"}
    recs = torch.cat(step.records, 0) if step.records else torch.zeros(0, 4)
    total_utts = info.world * B * args.steps
    value = total_utts / elapsed
    ok = float(recs[:, 2].mean()) if len(recs) else 0.0
    cmd_match = float((recs[:, 0] == recs[:, 1]).double().mean()) if len(recs) else 0.0
    e2e = stats["e2e_marginal_ms_per_added_command"]
    e2e = pdist.max_over_ranks(info, e2e if e2e is not None else -1.0)
    ref = stats["ref_equiv_ms_per_added_command"]
    ref = pdist.max_over_ranks(info, ref if ref is not None else -1.0)
    if info.is_main:
        out = {
            "metric": ("utterances_per_sec (multi-command utterances; ms per added command "
                       "reported alongside)"),
            "value": round(value, 3),
            "unit": "utterances/s",
            "n_gpus": info.world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": ("synthetic speech-like PCM16, every utterance a distinct transcript (no "
                     "repeated prompts) + random-init weights (teacher-forced STT, "
                     "grammar-constrained LLM)"),
            "config": {"model": f"{args.stt} + {args.llm}", "global_batch": info.world * B,
                       "seq_len": 1500, "parallelism": f"dp{info.world}",
                       "commands_mix": mix, "baseline_config": 4, "mode": args.mode,
                       "concurrent_streams_per_gpu": B,
                       "inflight": args.inflight if args.mode == "batch" else None},
            "ms_per_added_command_e2e_marginal": None if e2e < 0 else round(e2e, 3),
            "ms_per_added_command_ref_equiv": None if ref < 0 else round(ref, 4),
            "baseline_ms_per_added_command": BASELINE_MS_PER_ADDED_COMMAND,
            "added_command_speedup_vs_baseline": (None if e2e <= 0 else
                                                  round(BASELINE_MS_PER_ADDED_COMMAND / e2e, 3)),
            "queue_success_rate": round(ok, 4),
            "command_count_match_rate": round(cmd_match, 4),
            "phase_ms_per_step": phase_ms,
            "llm_stats": llm_stats_t,
            "stt_stats": stt_stats_t,
            "hub": hub_stats,
            "window_300ms": window,
            "fused_gemm_tuning": {f"{k[0]}:{k[1]}x{k[2]}:M{k[3]}": list(v)
                                  for k, v in ops._FSPLITS.items()},
            "init_s": round(t_init, 2),
        }
        print(json.dumps(out), flush=True)
    if hub is not None:
        relays.close()
        loop.run_until_complete(hub.stop())
    loop.run_until_complete(nats.close())
    pdist.shutdown(info)
    if broker is not None:
        broker.stdin.close()
        broker.wait(timeout=10)
    return 0


if __name__ == "__main__":
    sys.exit(main())
