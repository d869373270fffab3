"""GPU voice pipeline: batched STT -> ONE constrained multi-command parse per
utterance -> command queue (rollback) -> NATS publish -> voice-event record.

This is the MI355X replacement of the reference's winner path
(``audio_service.go:590-761``: transcribe, bridge / ParseMultiCommand, TTS,
NATS), restructured for batching: every stage runs once per *batch* of
arbitration winners on one GPU, and the command queue of each utterance runs
as soon as its own decode finishes.
"""
from __future__ import annotations

import asyncio
import time
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass, field

import numpy as np
import torch

from ..llm.command_queue import CommandQueue, ExecutionResult
from ..llm.commands import (Command, MultiCommand, ParseError, detect_compound_utterance,
                            parse_multi_command_response, parse_response,
                            split_compound_utterance)
from ..llm.prompts import build_multi_command_prompt, build_prompt
from ..llm.transcriber import TranscriptionResult, to_transcription_result
from ..transport.device_commands import ExecutionContext, NATSCommandExecutor
from ..utils.faults import faults
from ..utils.tracing import tracer
from .grammar import multi_command_schema, single_command_schema
from .llm_engine import GenRequest, LLMEngine
from .stt_engine import STTEngine, STTRequest


@dataclass
class PipelineJob:
    relay_id: str
    request_id: str
    pcm: np.ndarray
    # synthetic ground truth (teacher forcing); a list = one text per 30 s
    # window of a long-form utterance
    transcript_hint: str | list | None = None
    staged: object = None                  # pinned PCM slot with the samples (relay path)
    on_tokens: object = None               # streaming hook: called with each step's token ids
    # results
    transcription: TranscriptionResult | None = None
    raw_text: str = ""
    rms: float = 0.0
    multi: MultiCommand | None = None
    n_expected: int = 0
    llm_output: str = ""
    queue: ExecutionResult | None = None
    error: str = ""
    stt_failed: bool = False
    llm_steps: int = 0                      # decode steps the intent parse sampled in
    t: dict = field(default_factory=dict)   # stage timestamps (perf_counter)

    @property
    def n_commands(self) -> int:
        return len(self.multi.commands) if self.multi else 0


def _stt_request(j: PipelineJob) -> STTRequest:
    h = j.transcript_hint
    if isinstance(h, (list, tuple)):
        return STTRequest(j.pcm, transcript=" ".join(h), transcript_windows=list(h), staged=j.staged)
    return STTRequest(j.pcm, transcript=h, staged=j.staged)


class VoicePipeline:
    def __init__(self, stt: STTEngine, llm: LLMEngine, nats=None, *, min_response_tokens: int = 8,
                 queue_max_duration: float = 0.0, rollback: bool = True, tts=None,
                 response_audio: bool = False, overlap: bool = True,
                 continuous: bool | None = None, batch_window: float = 0.002,
                 max_batch: int = 8, stt_priority: int = -1,
                 stt_continuous: bool | None = None):
        self.stt, self.llm, self.nats = stt, llm, nats
        self.min_response_tokens = min_response_tokens
        self.queue_max_duration = queue_max_duration
        self.rollback = rollback
        self.tts = tts
        self.response_audio = response_audio
        # overlap: STT and the LLM decode run on their own worker threads and
        # HIP streams, so batch k+1's (compute-bound) encoder overlaps batch k's
        # (HBM-bound) decode when several batches are in flight
        self.overlap = overlap and llm.device.type == "cuda"
        # continuous: utterances join the LLM engine's running decode batch
        # (scheduler thread) instead of decoding batch by batch
        self.continuous = self.overlap if continuous is None else continuous
        self.batch_window, self.max_batch = batch_window, max_batch
        self.stt_priority = stt_priority
        # continuous STT: arrivals join the running Whisper decode batch
        self.stt_continuous = self.continuous if stt_continuous is None else stt_continuous
        self._pool: ThreadPoolExecutor | None = None
        self._stt_pool: ThreadPoolExecutor | None = None
        self._pending: list[tuple[PipelineJob, asyncio.Future]] = []
        self._batcher: asyncio.Task | None = None
        self._stt_lock: asyncio.Lock | None = None
        self.stats = {"stt_batches": 0, "utterances": 0}

    def warmup(self) -> dict:
        """Capture every decode graph bucket of both engines before serving
        (the two engines run on their own threads; no capture may happen
        while the other thread is issuing HIP calls)."""
        out = {"stt_graphs": 0, "llm_graphs": 0}
        if self.overlap:
            out["stt_graphs"] = self.stt.warmup_graphs()
            out["llm_graphs"] = self.llm.warmup_graphs()
            torch.cuda.synchronize(self.llm.device)
        return out

    # --------------------------------------------------------------- stages
    def transcribe(self, jobs: list[PipelineJob], device_pcm=None) -> None:
        if device_pcm is not None and device_pcm.is_cuda:
            # the samples were produced on the default stream (e.g. an RCCL scatter)
            cur = torch.cuda.current_stream(device_pcm.device)
            cur.wait_stream(torch.cuda.default_stream(device_pcm.device))
        reqs = [_stt_request(j) for j in jobs]
        self.stt.transcribe(reqs, device_pcm)
        for j, r in zip(jobs, reqs):
            self._stt_post(j, r)

    def _stt_post(self, j: PipelineJob, r: STTRequest) -> None:
        j.raw_text, j.rms = r.text, r.rms
        j.t["stt_done"] = time.perf_counter()
        if r.t_enc0:
            j.t["enc0"], j.t["enc1"], j.t["dec0"] = r.t_enc0, r.t_enc1, r.t_dec0
        fi = faults()
        if fi and fi.active("stt_error"):
            j.stt_failed, j.error = True, "stt: injected fault"
            return
        j.transcription = to_transcription_result(r.text)

    def build_request(self, j: PipelineJob) -> GenRequest | None:
        if j.stt_failed:
            return None
        text = j.transcription.text if j.transcription else ""
        fi = faults()
        if text and fi and fi.active("llm_timeout"):
            j.error = "llm: injected timeout"   # -> parse-failed reply, no commands
            return None
        if not text:
            j.multi = MultiCommand([], False, text, "I didn't hear anything.")
            return None
        tok = self.llm.tok
        if detect_compound_utterance(text):
            n = max(1, len(split_compound_utterance(text)))
            j.n_expected = n
            prompt = build_multi_command_prompt(text)
            schema = multi_command_schema(n, min_response_tokens=self.min_response_tokens)
            r = GenRequest(tok.encode_prompt(prompt), schema, on_tokens=j.on_tokens)
            r.kind = "multi"  # type: ignore[attr-defined]
        else:
            j.n_expected = 1
            schema = single_command_schema(max_response_tokens=12)
            r = GenRequest(tok.encode_prompt(build_prompt(text)), schema, on_tokens=j.on_tokens)
            r.kind = "single"  # type: ignore[attr-defined]
        return r

    def parse(self, j: PipelineJob, r: GenRequest) -> None:
        text = j.transcription.text
        j.llm_output = r.output
        try:
            if getattr(r, "kind", "multi") == "multi":
                j.multi = parse_multi_command_response(r.output, text)
            else:
                cmd = parse_response(r.output)
                j.multi = MultiCommand([cmd], False, text, cmd.response)
        except ParseError as e:
            j.error = str(e)
            j.multi = MultiCommand([Command("unknown", {}, 0.0, "I'm not sure what you want me to do.")],
                                   False, text, "I'm not sure what you want me to do.")

    async def execute(self, j: PipelineJob) -> None:
        if not j.multi or not j.multi.commands:
            return
        ctx = ExecutionContext(j.relay_id, j.request_id, "", j.transcription.text)
        q = CommandQueue(j.multi.commands, self.queue_max_duration, self.rollback)
        with tracer().span("queue", request=j.request_id, commands=len(j.multi.commands)):
            j.queue = await q.execute(NATSCommandExecutor(self.nats, ctx))
        j.t["queue_done"] = time.perf_counter()

    # ------------------------------------------------------------- batch run
    def _worker(self, name: str, own_stream: bool, priority: int = 0) -> ThreadPoolExecutor:
        dev = self.llm.device

        def init():
            if dev.type == "cuda":
                torch.cuda.set_device(dev)
                if own_stream:
                    torch.cuda.set_stream(torch.cuda.Stream(dev, priority=priority))
        return ThreadPoolExecutor(1, thread_name_prefix=name, initializer=init)

    def _gpu_executor(self) -> ThreadPoolExecutor:
        if self._pool is None:
            self._pool = self._worker("gpu-worker", self.overlap)
        return self._pool

    def _stt_executor(self) -> ThreadPoolExecutor:
        if not self.overlap:
            return self._gpu_executor()
        if self._stt_pool is None:
            # the Whisper decoder is a latency-bound chain of small launches:
            # on a high-priority queue its workgroups are dispatched ahead of
            # the concurrent (bandwidth-bound) LLM decode GEMMs
            self._stt_pool = self._worker("stt-worker", True, self.stt_priority)
        return self._stt_pool

    # ------------------------------------------------------------ serving
    async def submit(self, job: PipelineJob) -> PipelineJob:
        """Serve one utterance. Arrivals are micro-batched for the STT stage
        (every utterance that arrived while the previous STT batch ran, up to
        ``max_batch``); their parses then join the LLM engine's running decode
        batch, and each command queue starts as soon as its own decode ends."""
        loop = asyncio.get_running_loop()
        fut = loop.create_future()
        self._pending.append((job, fut))
        if self._batcher is None or self._batcher.done():
            self._batcher = loop.create_task(self._batch_loop())
        return await fut

    async def _batch_loop(self) -> None:
        if self._stt_lock is None:
            self._stt_lock = asyncio.Lock()
        while self._pending:
            await asyncio.sleep(self.batch_window)
            batch = self._pending[: self.max_batch]
            self._pending = self._pending[self.max_batch:]
            if self.stt_continuous:
                self._submit_stt(batch)
                continue
            async with self._stt_lock:
                jobs = [j for j, _ in batch]
                try:
                    await self._stt_stage(jobs)
                except Exception as e:  # noqa: BLE001
                    for j, f in batch:
                        if not f.done():
                            f.set_exception(e)
                    continue
            asyncio.ensure_future(self._finish(batch))

    def _submit_stt(self, batch) -> None:
        """Continuous STT: the micro-batch joins the STT engine's running
        decoder batch (no wait for an earlier batch to drain) and every
        utterance moves on to the LLM the moment its OWN transcript is done."""
        loop = asyncio.get_running_loop()
        t0 = time.perf_counter()
        reqs = []
        owner = {}
        for j, f in batch:
            j.t["start"] = j.t.get("start", t0)
            r = _stt_request(j)
            reqs.append(r)
            owner[id(r)] = (j, f)
        self.stats["stt_batches"] += 1
        self.stats["utterances"] += len(reqs)

        def start_llm(r: STTRequest) -> None:
            j, f = owner[id(r)]
            self._stt_post(j, r)
            asyncio.ensure_future(self._finish([(j, f)]))

        def on_stt_done(r: STTRequest) -> None:      # STT scheduler thread
            loop.call_soon_threadsafe(start_llm, r)

        self.stt.start(self.stt_priority)
        fut = self.stt.submit_batch(reqs, on_stt_done)

        def failed(ft) -> None:
            e = ft.exception()
            if e is None:
                return

            def fail():
                for j, f in batch:
                    if not f.done():
                        f.set_exception(e)
            loop.call_soon_threadsafe(fail)
        fut.add_done_callback(failed)

    async def _finish(self, batch) -> None:
        futs = {id(j): f for j, f in batch}

        def job_done(j: PipelineJob) -> None:  # each reply as soon as ITS queue is done
            f = futs.get(id(j))
            if f is not None and not f.done():
                f.set_result(j)
        try:
            await self._llm_stage([j for j, _ in batch], job_done)
        except Exception as e:  # noqa: BLE001
            for _, f in batch:
                if not f.done():
                    f.set_exception(e)
            return
        for j, f in batch:
            if not f.done():
                f.set_result(j)

    async def process(self, jobs: list[PipelineJob], device_pcm=None) -> list[PipelineJob]:
        """One batch end to end: STT on the STT worker thread, then the LLM
        stage; each utterance's command queue is scheduled on the event loop
        the moment its own decode finishes, so command execution / NATS
        publishing overlaps the remaining decode."""
        await self._stt_stage(jobs, device_pcm)
        await self._llm_stage(jobs)
        return jobs

    async def _stt_stage(self, jobs: list[PipelineJob], device_pcm=None) -> None:
        loop = asyncio.get_running_loop()
        t0 = time.perf_counter()
        for j in jobs:
            j.t["start"] = j.t.get("start", t0)
        await loop.run_in_executor(self._stt_executor(), self.transcribe, jobs, device_pcm)
        self.stats["stt_batches"] += 1
        self.stats["utterances"] += len(jobs)

    async def _llm_stage(self, jobs: list[PipelineJob], job_done=None) -> None:
        loop = asyncio.get_running_loop()
        reqs, owners = [], []
        for j in jobs:
            r = self.build_request(j)
            if r is not None:
                reqs.append(r)
                owners.append(j)
            elif job_done is not None:
                job_done(j)
        owner_of = {id(r): j for r, j in zip(reqs, owners)}
        tasks: list[asyncio.Future] = []

        t_llm = time.monotonic()

        def start_queue(r: GenRequest) -> None:
            j = owner_of[id(r)]
            # per-utterance LLM span (submit -> its own decode done): replies go
            # out per utterance, so a batch-level span could outlive the caller
            tracer().record("llm", t_llm, time.monotonic(), request=j.request_id)
            j.t["llm_first"] = r.t_first
            j.t["llm_done"] = r.t_done
            j.llm_steps = r.steps
            with tracer().span("parse", request=j.request_id):
                self.parse(j, r)
            t = asyncio.ensure_future(self.execute(j))
            if job_done is not None:
                t.add_done_callback(lambda _t, j=j: job_done(j))
            tasks.append(t)

        def on_done(r: GenRequest) -> None:  # called on the GPU worker thread
            loop.call_soon_threadsafe(start_queue, r)

        if reqs:
            if self.continuous:
                await asyncio.wrap_future(self.llm.submit_batch(reqs, on_done))
            else:
                await loop.run_in_executor(self._gpu_executor(), self.llm.generate, reqs, on_done)
        await asyncio.sleep(0)  # let the last call_soon_threadsafe callbacks run
        while len(tasks) < len(reqs):
            await asyncio.sleep(0.0005)
        await asyncio.gather(*tasks)


def added_command_stats(jobs: list[PipelineJob]) -> dict:
    """Both BASELINE.md definitions of 'ms per added command':
    * reference-equivalent: queue item durations for index >= 1
      (command_queue.go:119-121: execution + NATS publish);
    * end-to-end marginal: slope of (utterance completion latency) vs
      (number of commands) across the batch (decode tokens + execution)."""
    added = [it.duration * 1e3 for j in jobs if j.queue for it in j.queue.completed_items if it.index >= 1]
    xs, ys = [], []
    for j in jobs:
        if j.queue is not None and "queue_done" in j.t:
            xs.append(j.n_commands)
            ys.append((j.t["queue_done"] - j.t["start"]) * 1e3)
    slope = None
    if len(set(xs)) >= 2:
        slope = float(np.polyfit(np.array(xs, float), np.array(ys, float), 1)[0])
    return {"ref_equiv_ms_per_added_command": float(np.mean(added)) if added else None,
            "ref_equiv_ms_per_added_command_max": float(np.max(added)) if added else None,
            "e2e_marginal_ms_per_added_command": slope,
            "n_added_commands": len(added)}
