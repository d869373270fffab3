"""Served-hub FRONT END under BASELINE config-4 load, without GPUs (VERDICT
r4 #7): the real front end (``HubServer``: grpc.aio AudioService with
per-group arbitration windows, the DP router, the shared-memory PCM ring,
SQLite voice events) over N stub worker processes (``parallel/stub_worker.py``:
fixed-latency fake GPU), driven by R concurrent relays from separate client
processes. Each relay loops StreamAudio calls: a wake-word chunk, then the
speech as 100 ms chunks (3200 B), end of speech on the last.

Reports sustained utterances/s and the latency the front end ADDS over the
arbitration window and the fake GPU time (p50 / p99). ``--paced``: the
relays send their chunks in real time (one 100 ms chunk per 100 ms).

    python scripts/frontend_bench.py --relays 64 --workers 8 --seconds 20
"""
import argparse
import asyncio
import json
import multiprocessing as mp
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _client_proc(port: int, relays: list[int], t_end: float, paced: bool, warm_s: float,
                 out_q) -> None:
    import grpc

    from loqa_hub_amd.engine.synthetic import make_utterance
    from loqa_hub_amd.transport.audio_proto import AudioChunk, stream_audio_stub
    utts = [make_utterance(3, i, 1 + i % 4) for i in range(16)]
    datas = [np.ascontiguousarray(u.pcm, dtype="<i2").tobytes() for u in utts]

    async def main():
        recs = []
        async with grpc.aio.insecure_channel(f"127.0.0.1:{port}") as ch:
            call = stream_audio_stub(ch)

            async def relay(ci: int) -> None:
                k = 0
                while time.time() < t_end:
                    data = datas[(ci + k) % len(datas)]
                    k += 1
                    wake, rest = data[:9600], data[9600:]

                    async def chunks():
                        yield AudioChunk(relay_id=f"relay-{ci}", audio_data=wake, sample_rate=16000,
                                         is_wake_word=True)
                        for o in range(0, len(rest), 3200):
                            if paced:
                                await asyncio.sleep(0.1)
                            yield AudioChunk(relay_id=f"relay-{ci}", audio_data=rest[o:o + 3200],
                                             sample_rate=16000,
                                             is_end_of_speech=o + 3200 >= len(rest))
                    t0 = time.time()
                    got = [r async for r in call(chunks())]
                    t1 = time.time()
                    speech = (len(rest) // 3200) * 0.1 if paced else 0.0
                    recs.append((t0, t1, (t1 - t0) - speech, bool(got) and got[-1].success))
            await asyncio.gather(*[relay(ci) for ci in relays])
        out_q.put(recs)
    asyncio.run(main())


def run(relays: int = 64, workers: int = 8, seconds: float = 20.0, window_ms: float = 300.0,
        gpu_ms: float = 50.0, paced: bool = False, client_procs: int = 4, warm_s: float = 3.0,
        bypass: bool = False, shm_slots: int | None = None) -> dict:
    from loqa_hub_amd import config as cfgmod
    from loqa_hub_amd.server import HubServer, build_dp_processor
    if shm_slots is not None:
        from loqa_hub_amd.parallel import dp_serving
        dp_serving.SHM_SLOTS = shm_slots
    tmp = tempfile.mkdtemp(prefix="loqa-fe-")
    env = {"LOQA_DB_PATH": os.path.join(tmp, "hub.db"), "NATS_URL": "embedded",
           "ARBITRATION_SCOPE": "per_relay_group",
           "ARBITRATION_WINDOW_DURATION": f"{window_ms}ms",
           "HUB_TTS_BACKEND": "none", "STREAMING_ENABLED": "false"}
    if bypass:
        env["ARBITRATION_SINGLE_RELAY_BYPASS"] = "true"
    cfg = cfgmod.load(env)

    async def main() -> dict:
        srv = HubServer(cfg, skills_dir=os.path.join(tmp, "skills"),
                        skills_config_store=os.path.join(tmp, "skillcfg"),
                        transcript_hints=lambda relay: "turn on the lights")
        await srv._connect_nats()
        from loqa_hub_amd.parallel.stub_worker import stub_factory
        srv.processor = await build_dp_processor(cfg, workers, srv.nats.url, device="cpu",
                                                 factory=stub_factory, stub_gpu_ms=gpu_ms,
                                                 heartbeat_s=0.5)
        await srv.start(host="127.0.0.1", http_port=0, grpc_port=0)
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        t_start = time.time() + 2.0                  # client start-up (imports)
        t_end = t_start + warm_s + seconds
        groups = [list(range(relays))[i::client_procs] for i in range(client_procs)]
        procs = [ctx.Process(target=_client_proc, args=(srv.grpc_port, g, t_end, paced, warm_s, q))
                 for g in groups]
        for p in procs:
            p.start()
        recs = []
        try:
            while len(recs) < len(procs):
                try:
                    recs.append(await asyncio.to_thread(q.get, True, seconds + warm_s + 120))
                except Exception:
                    break
            stats = dict(srv.audio_service.stats)
            dpst = srv.processor.stats
        finally:
            for p in procs:
                p.join(timeout=30)
                if p.is_alive():
                    p.kill()
            await srv.stop()
        return {"recs": [r for rr in recs for r in rr], "svc": stats, "dp": dpst}
    res = asyncio.run(main())
    recs = sorted(res["recs"])
    if not recs:
        raise RuntimeError("no utterances completed")
    t_first = recs[0][0]
    lo = t_first + warm_s
    meas = [r for r in recs if r[0] >= lo]
    t_hi = max(r[1] for r in meas)
    dur = t_hi - lo
    base = (0.0 if bypass else window_ms / 1e3) + gpu_ms / 1e3
    added = np.array([(r[2] - base) * 1e3 for r in meas])
    ok = float(np.mean([r[3] for r in meas]))
    return {"relays": relays, "workers": workers, "window_ms": window_ms, "stub_gpu_ms": gpu_ms,
            "paced": paced, "bypass": bypass, "measured_s": round(dur, 2),
            "utterances": len(meas), "utt_per_s": round(len(meas) / dur, 1),
            "ideal_utt_per_s": round(relays / base, 1) if not paced else None,
            "added_ms_p50": round(float(np.percentile(added, 50)), 2),
            "added_ms_p99": round(float(np.percentile(added, 99)), 2),
            "added_ms_max": round(float(added.max()), 2), "success_rate": ok,
            "pcm_shm_sent": res["dp"].get("pcm_shm_sent"),
            "pcm_inline_sent": res["dp"].get("pcm_inline_sent"),
            "svc": res["svc"]}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--relays", type=int, default=64)
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--seconds", type=float, default=20.0)
    ap.add_argument("--window-ms", type=float, default=300.0)
    ap.add_argument("--gpu-ms", type=float, default=50.0)
    ap.add_argument("--paced", action="store_true")
    ap.add_argument("--bypass", action="store_true")
    ap.add_argument("--client-procs", type=int, default=4)
    ap.add_argument("--shm-slots", type=int, default=None, help="0: PCM as pickled bytes")
    a = ap.parse_args()
    print(json.dumps(run(a.relays, a.workers, a.seconds, a.window_ms, a.gpu_ms, a.paced,
                         a.client_procs, bypass=a.bypass, shm_slots=a.shm_slots)))
    return 0


if __name__ == "__main__":
    sys.exit(main())
