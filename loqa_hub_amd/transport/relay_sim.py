"""Relay simulator: B relay devices as closed loops of gRPC ``StreamAudio``
calls, in a process of their own (as real relays are separate devices).

Each relay sends a wake-word chunk (300 ms of PCM16), then 100 ms chunks, the
last one flagged end-of-speech (``audio_service.go:926-1043`` is the server
side), waits for the hub's response and starts its next utterance. The
utterances are the bench's distinct synthetic ones (``engine/synthetic.py``
``make_unique``), drawn from the same seed as the hub process, which keeps the
matching transcripts as teacher-forcing hints (random-init Whisper).

Keeping the relays out of the hub's process matters for a served benchmark:
in one process, the relays' protobuf encoding and gRPC client work share the
GIL with the hub's scheduler threads.

Protocol (line-based, stdin -> stdout): ``run <base> <n>`` runs every relay
for ``n`` utterances starting at index ``base`` of its list and answers
``done <json>`` with per-relay ``[expected commands, ok, latency ms, request
id]`` records; ``counts`` answers the commands published per request id on
``loqa.voice.commands`` (observed over NATS); ``quit`` exits. The first line
printed is ``ready``.

    python -m loqa_hub_amd.transport.relay_sim --port P --nats URL --rank R \\
        --relays B --seed S --mix 1,2,3,4 --per-relay N [--paced]
"""
from __future__ import annotations

import argparse
import asyncio
import json
import sys
import time

import numpy as np

from ..engine.synthetic import make_unique

WAKE_BYTES = 9600          # 300 ms of 16 kHz PCM16
CHUNK_BYTES = 3200         # 100 ms


def relay_name(rank: int, ci: int) -> str:
    return f"relay-{rank}-{ci}"


def relay_utterances(seed: int, mix: list[int], relays: int, per_relay: int, rank: int = 0):
    """Every relay's utterance list (the hub process draws the same)."""
    counts = [mix[(ci + k) % len(mix)] for ci in range(relays) for k in range(per_relay)]
    uniq = make_unique(seed, counts, offset=rank * relays * per_relay)
    return [uniq[ci * per_relay:(ci + 1) * per_relay] for ci in range(relays)]


async def _serve(a) -> None:
    import grpc

    from ..messaging.nats_client import NATSClient
    from .audio_proto import AudioChunk, stream_audio_stub
    mix = [int(x) for x in a.mix.split(",")]
    utts = relay_utterances(a.seed, mix, a.relays, a.per_relay, a.rank)
    per_request: dict[str, int] = {}
    nc = NATSClient(name=f"relay-sim-{a.rank}")
    await nc.connect(a.nats)

    def on_msg(m):
        rid = json.loads(m.data).get("request_id", "")
        per_request[rid] = per_request.get(rid, 0) + 1
    await nc.subscribe("loqa.voice.commands", on_msg)
    await nc.flush()
    ch = grpc.aio.insecure_channel(f"127.0.0.1:{a.port}")
    call = stream_audio_stub(ch)

    async def relay(ci: int, base: int, n: int, out: list) -> None:
        name = relay_name(a.rank, ci)
        for k in range(base, base + n):
            u = utts[ci][k]
            data = np.ascontiguousarray(u.pcm, dtype="<i2").tobytes()
            wake, rest = data[:WAKE_BYTES], data[WAKE_BYTES:]

            async def chunks():
                yield AudioChunk(relay_id=name, audio_data=wake, sample_rate=16000, is_wake_word=True)
                for o in range(0, max(len(rest), 1), CHUNK_BYTES):
                    if a.paced:                    # a real relay: one 100 ms chunk per 100 ms
                        await asyncio.sleep(CHUNK_BYTES / 32000)
                    yield AudioChunk(relay_id=name, audio_data=rest[o:o + CHUNK_BYTES],
                                     sample_rate=16000, is_end_of_speech=o + CHUNK_BYTES >= len(rest))
            t0 = time.perf_counter()
            got = [r async for r in call(chunks())]
            lat = (time.perf_counter() - t0) * 1e3
            if a.paced:                            # latency after the relay stopped speaking
                lat -= 1e3 * (-(-max(len(rest), 1) // CHUNK_BYTES)) * CHUNK_BYTES / 32000
            ok = bool(got) and got[-1].success
            rid = got[-1].request_id if got else ""
            out.append([name, u.n_commands, float(ok), lat, rid])

    loop = asyncio.get_running_loop()
    reader = asyncio.StreamReader()
    await loop.connect_read_pipe(lambda: asyncio.StreamReaderProtocol(reader), sys.stdin)
    print("ready", flush=True)
    while True:
        line = (await reader.readline()).decode().split()
        if not line or line[0] == "quit":
            break
        if line[0] == "run":
            base, n = int(line[1]), int(line[2])
            out: list = []
            await asyncio.gather(*[relay(ci, base, n, out) for ci in range(a.relays)])
            print("done " + json.dumps(out), flush=True)
        elif line[0] == "counts":
            await nc.flush()
            await asyncio.sleep(0.2)
            print("counts " + json.dumps(per_request), flush=True)
    await ch.close()
    await nc.close()


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--port", type=int, required=True)
    ap.add_argument("--nats", required=True)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--relays", type=int, default=8)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--mix", default="1,2,3,4")
    ap.add_argument("--per-relay", type=int, required=True)
    ap.add_argument("--paced", action="store_true")
    asyncio.run(_serve(ap.parse_args(argv)))
    return 0


class RelayProcess:
    """Hub-side handle of a relay simulator subprocess."""

    def __init__(self, *, port: int, nats_url: str, rank: int, relays: int, seed: int, mix: str,
                 per_relay: int, paced: bool = False, cwd: str | None = None):
        import subprocess
        cmd = [sys.executable, "-m", "loqa_hub_amd.transport.relay_sim", "--port", str(port),
               "--nats", nats_url, "--rank", str(rank), "--relays", str(relays), "--seed", str(seed),
               "--mix", mix, "--per-relay", str(per_relay)] + (["--paced"] if paced else [])
        self.p = subprocess.Popen(cmd, stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True,
                                  cwd=cwd)
        self._expect("ready")

    def _expect(self, word: str) -> str:
        line = self.p.stdout.readline()
        if not line.startswith(word):
            self.close()
            raise RuntimeError(f"relay simulator: expected {word!r}, got {line[:200]!r}")
        return line[len(word):].strip()

    def _send(self, cmd: str) -> None:
        self.p.stdin.write(cmd + "\n")
        self.p.stdin.flush()

    async def run(self, base: int, n: int) -> list:
        """Every relay's utterances [base, base + n); per-utterance records
        [relay, expected commands, ok, latency ms, request id]."""
        self._send(f"run {base} {n}")
        return json.loads(await asyncio.to_thread(self._expect, "done"))

    async def counts(self) -> dict:
        self._send("counts")
        return json.loads(await asyncio.to_thread(self._expect, "counts"))

    def close(self) -> None:
        if self.p.poll() is None:
            try:
                self._send("quit")
                self.p.wait(timeout=10)
            except Exception:  # noqa: BLE001
                self.p.kill()


if __name__ == "__main__":
    sys.exit(main())
