"""Progressive TTS pipeline (``internal/llm/streaming_audio_pipeline.go``).

Per session: phrase processor -> synthesis queue (20) -> N workers (default 3)
-> completed jobs (20) -> sequencer that re-orders by sequence id through a
pending map (:106-399). A closed phrase stream enqueues an empty "end" job that
becomes the ``is_last`` chunk. Metrics use the reference's pairwise moving
average for synthesis time.

Deliberate fix: the reference emits the last chunk as soon as *a* worker picks
up the end sentinel, which can overtake still-synthesising phrases; here the end
marker carries the next sequence id and is released by the sequencer only after
every earlier phrase has been delivered (or failed).

The TTS backend is any ``TextToSpeech``: the on-GPU VITS engine (phrases of
concurrent sessions batch into one GPU call) or the OpenAI-compatible client.
"""
from __future__ import annotations

import asyncio
import time
from dataclasses import dataclass, field

from ..llm.tts import TextToSpeech, TTSOptions, TTSResult
from .chan import Chan, ChannelClosed


@dataclass
class AudioChunk:
    audio: bytes = b""
    content_type: str = ""
    length: int = 0
    sequence_id: int = 0
    is_last: bool = False
    phrase: str = ""
    timestamp: float = 0.0


@dataclass
class SynthesisJob:
    id: int
    phrase: str
    options: TTSOptions | None
    start_time: float = 0.0
    completed_at: float = 0.0
    result: TTSResult | None = None
    error: Exception | None = None


@dataclass
class PipelineMetrics:
    start_time: float = 0.0
    first_audio_time: float = 0.0
    total_phrases: int = 0
    synthesized_phrases: int = 0
    failed_synthesis: int = 0
    average_synthesis_time: float = 0.0
    total_audio_duration: float = 0.0
    queue_high_water_mark: int = 0


@dataclass
class PipelineContext:
    id: str
    audio_chunks: Chan = field(default_factory=lambda: Chan(10))
    errors: Chan = field(default_factory=lambda: Chan(5))
    metrics: PipelineMetrics = field(default_factory=PipelineMetrics)
    synthesis_queue: Chan = field(default_factory=lambda: Chan(20))
    completed_jobs: Chan = field(default_factory=lambda: Chan(20))
    tasks: list = field(default_factory=list)

    def cancel(self) -> None:
        for t in self.tasks:
            if not t.done():
                t.cancel()


class StreamingAudioPipeline:
    def __init__(self, tts: TextToSpeech, options: TTSOptions | None = None,
                 max_concurrent: int = 3):
        self.tts = tts
        self.options = options or TTSOptions("af_bella", 1.0, "wav", True)
        self.max_concurrent = max_concurrent
        self.active: dict[str, PipelineContext] = {}

    def start_pipeline(self, context_id: str, phrases: Chan) -> PipelineContext:
        if context_id in self.active:
            raise ValueError(f"pipeline context {context_id} already exists")
        pc = PipelineContext(context_id, metrics=PipelineMetrics(start_time=time.monotonic()))
        self.active[context_id] = pc
        loop = asyncio.get_running_loop()
        pc.tasks = [loop.create_task(self._phrase_processor(pc, phrases)),
                    loop.create_task(self._worker_pool(pc)),
                    loop.create_task(self._sequencer(pc))]
        return pc

    async def stop_pipeline(self, context_id: str) -> None:
        pc = self.active.pop(context_id, None)
        if pc is None:
            return
        pc.cancel()
        await asyncio.gather(*pc.tasks, return_exceptions=True)
        pc.audio_chunks.close()
        pc.errors.close()

    async def _phrase_processor(self, pc: PipelineContext, phrases: Chan) -> None:
        seq = 0
        try:
            async for phrase in phrases:
                if not phrase:
                    continue
                pc.metrics.total_phrases += 1
                pc.metrics.queue_high_water_mark = max(pc.metrics.queue_high_water_mark,
                                                       len(pc.synthesis_queue))
                await pc.synthesis_queue.put(SynthesisJob(seq, phrase, self.options,
                                                          time.monotonic()))
                seq += 1
            await pc.synthesis_queue.put(SynthesisJob(seq, "", self.options, time.monotonic()))
        finally:
            pc.synthesis_queue.close()

    async def _worker_pool(self, pc: PipelineContext) -> None:
        try:
            await asyncio.gather(*[self._worker(pc) for _ in range(max(1, self.max_concurrent))])
        finally:
            pc.completed_jobs.close()

    async def _worker(self, pc: PipelineContext) -> None:
        async for job in pc.synthesis_queue:
            if job.phrase == "":
                job.completed_at = time.monotonic()
                await pc.completed_jobs.put(job)
                continue
            try:
                job.result = await self.tts.synthesize(job.phrase, job.options)
            except Exception as e:  # noqa: BLE001
                job.error = e
            job.completed_at = time.monotonic()
            m = pc.metrics
            if job.error is not None:
                m.failed_synthesis += 1
                pc.errors.try_put(RuntimeError(f"TTS synthesis failed for job {job.id}: {job.error}"))
            else:
                m.synthesized_phrases += 1
                dt = job.completed_at - job.start_time
                m.average_synthesis_time = dt if m.average_synthesis_time == 0 else \
                    (m.average_synthesis_time + dt) / 2
            await pc.completed_jobs.put(job)

    async def _sequencer(self, pc: PipelineContext) -> None:
        pending: dict[int, SynthesisJob] = {}
        nxt = 0
        try:
            async for job in pc.completed_jobs:
                pending[job.id] = job
                while nxt in pending:
                    j = pending.pop(nxt)
                    nxt += 1
                    if j.phrase == "":
                        await pc.audio_chunks.put(AudioChunk(sequence_id=j.id, is_last=True,
                                                             timestamp=time.monotonic()))
                        return
                    if j.error is None and j.result is not None:
                        if not pc.metrics.first_audio_time:
                            pc.metrics.first_audio_time = time.monotonic()
                        await pc.audio_chunks.put(AudioChunk(
                            j.result.audio, j.result.content_type, j.result.length, j.id, False,
                            j.phrase, time.monotonic()))
        except ChannelClosed:
            return

    def get_pipeline_metrics(self, context_id: str) -> PipelineMetrics:
        pc = self.active.get(context_id)
        if pc is None:
            raise KeyError(f"pipeline context {context_id} not found")
        return PipelineMetrics(**vars(pc.metrics))

    def get_active_pipelines(self) -> list[str]:
        return list(self.active)

    def update_tts_options(self, options: TTSOptions) -> None:
        self.options = options
