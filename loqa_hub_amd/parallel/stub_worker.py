"""A fixed-latency stand-in for a GPU worker's processor, for front-end load
tests of the served DP hub (``scripts/frontend_bench.py``,
``tests/test_frontend_load.py``): it receives the PCM exactly as a GPU worker
does (shared-memory ring slot or inline bytes), touches every sample (the RMS
the STT front end would compute), waits ``stub_gpu_ms`` as if the pipeline
ran, and answers with the teacher-forcing transcript, so the front end's own
cost - gRPC chunks, arbitration windows, routing, the PCM hand-off, SQLite
voice events - is what a run measures."""
from __future__ import annotations

import asyncio

import numpy as np

from ..transport.audio_service import UtteranceResult


class StubGPUProcessor:
    takes_pcm16 = True

    def __init__(self, spec: dict):
        self.rank = spec["rank"]
        self.delay = float(spec.get("stub_gpu_ms", 50.0)) / 1e3
        self.stats = {"utterances": 0, "samples": 0}

    async def process(self, relay_id, request_id, audio, sample_rate, transcript_hint=None,
                      pcm16=None, pcm_slot=None):
        x = pcm_slot.numpy() if pcm_slot is not None else pcm16
        n = int(x.size) if x is not None else 0
        rms = float(np.sqrt(np.mean(np.square(x, dtype=np.float64)))) / 32767 if n else 0.0
        await asyncio.sleep(self.delay)
        self.stats["utterances"] += 1
        self.stats["samples"] += n
        return UtteranceResult(transcription=transcript_hint or "", response_text="ok",
                               intents=["turn_on"], confidence=0.9 if rms >= 0 else 0.0)


def stub_factory(spec: dict, device: str) -> StubGPUProcessor:
    return StubGPUProcessor(spec)
