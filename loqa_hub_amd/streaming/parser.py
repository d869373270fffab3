"""Token-streaming command parser (``internal/llm/streaming_command_parser.go``).

A producer task fans tokens out to ``visual_tokens`` (cap 100), ``token_stream``
(100) and phrase-buffered ``audio_phrases`` (10), then delivers the parsed
``final_command`` (1) or an error on ``errors`` (1) (:45-53, :127-292).

Token sources (``StreamingBackend``):
* ``OllamaStreamingBackend`` - ``POST /api/generate`` with ``stream: true``,
  ``Accept: application/x-ndjson``; one JSON object per line (:339-385);
* ``GPUStreamingBackend``    - the on-device grammar-constrained decode; each
  engine step's emitted tokens (sampled + jump-forward) are pushed as they are
  produced, so the first visual token arrives after one decode step.

``PhraseBuffer`` flushes on the reference's boundary suffixes, at 50 tokens or
after 2 s since the last flush (:112-124, :295-336), but tests the suffix on a
bounded tail instead of re-joining the whole buffer per token (SURVEY §3.7 #10:
O(1) per token instead of O(n)).

Disabled mode answers through the non-streaming ``CommandParser`` as a single
token/phrase (:422-454); an empty transcription yields "I didn't hear anything.".
"""
from __future__ import annotations

import asyncio
import json
import logging
import time
from dataclasses import dataclass
from typing import AsyncIterator, Protocol

from ..llm.command_parser import CommandParser
from ..llm.commands import Command, parse_response
from ..llm.http import AiohttpClient, HTTPClient
from ..llm.prompts import build_streaming_prompt
from .chan import Chan, ChannelClosed

log = logging.getLogger("loqa.streaming")

BOUNDARIES = (".", "!", "?", ", and", ", then", ", so", ", but", ", however", ", because", "\n")
_TAIL = max(len(b) for b in BOUNDARIES)


@dataclass
class StreamingMetrics:
    start_time: float = 0.0
    first_token_time: float = 0.0
    first_phrase_time: float = 0.0
    completion_time: float = 0.0
    token_count: int = 0
    phrase_count: int = 0
    buffer_overflows: int = 0
    interrupt_count: int = 0


class PhraseBuffer:
    def __init__(self, max_buffer_time: float = 2.0, max_tokens: int = 50,
                 boundaries: tuple[str, ...] = BOUNDARIES):
        self.tokens: list[str] = []
        self.boundaries = boundaries
        self.tail_len = max(len(b) for b in boundaries)
        self.max_buffer_time = max_buffer_time
        self.max_tokens = max_tokens
        self.last_flush = 0.0
        self._tail = ""

    def add_token(self, token: str) -> str:
        self.tokens.append(token)
        self._tail = (self._tail + token)[-self.tail_len:]
        if any(self._tail.endswith(b) for b in self.boundaries):
            return self.flush()
        if len(self.tokens) >= self.max_tokens or (
                self.last_flush and time.monotonic() - self.last_flush >= self.max_buffer_time):
            return self.flush()
        return ""

    def flush(self) -> str:
        if not self.tokens:
            return ""
        phrase = "".join(self.tokens)
        self.tokens.clear()
        self._tail = ""
        self.last_flush = time.monotonic()
        return phrase.strip()


class StreamingResult:
    def __init__(self):
        self.token_stream = Chan(100)
        self.final_command = Chan(1)
        self.errors = Chan(1)
        self.visual_tokens = Chan(100)
        self.audio_phrases = Chan(10)
        self.metrics = StreamingMetrics(start_time=time.monotonic())
        self._task: asyncio.Task | None = None
        self.cancelled = asyncio.Event()

    def cancel(self) -> None:
        self.cancelled.set()
        if self._task is not None and not self._task.done():
            self._task.cancel()

    def close_outputs(self) -> None:
        for ch in (self.token_stream, self.final_command, self.visual_tokens, self.audio_phrases):
            ch.close()

    async def collect(self) -> tuple[list[str], list[str], Command | None, Exception | None]:
        """Drain everything (tests / non-interactive callers)."""
        toks, phrases = [], []

        async def drain(ch, out):
            async for v in ch:
                out.append(v)
        await asyncio.gather(drain(self.token_stream, toks), drain(self.audio_phrases, phrases),
                             drain(self.visual_tokens, []))
        cmd, _ = self.final_command.try_get()
        err, _ = self.errors.try_get()
        return toks, phrases, cmd, err


class StreamingBackend(Protocol):
    def stream(self, prompt: str) -> AsyncIterator[tuple[str, bool]]: ...


class OllamaStreamingBackend:
    def __init__(self, url: str, model: str, client: HTTPClient | None = None,
                 timeout: float = 30.0):
        self.url, self.model = url.rstrip("/"), model
        self.client = client or AiohttpClient()
        self.timeout = timeout

    async def stream(self, prompt: str):
        body = json.dumps({"model": self.model, "prompt": prompt, "stream": True}).encode()
        async for raw in self.client.stream_lines(
                "POST", self.url + "/api/generate", body=body,
                headers={"Content-Type": "application/json", "Accept": "application/x-ndjson"},
                timeout=self.timeout):
            line = raw.decode(errors="replace").strip() if isinstance(raw, bytes) else raw.strip()
            if not line:
                continue
            try:
                obj = json.loads(line)
            except ValueError as e:
                log.warning("failed to parse streaming line: %s", e)
                continue
            yield str(obj.get("response", "")), bool(obj.get("done", False))


class GPUStreamingBackend:
    """Streams the grammar-constrained decode of the local engine. Each prompt
    joins the engine's RUNNING continuous batch (``LLMEngine.submit_batch``)
    and its tokens are pushed as every decode step emits them, so streaming
    sessions share the decode steps (and their weight reads) with every other
    live sequence instead of running a blocking decode of their own. Engines
    without a scheduler (CPU tests) fall back to ``generate`` in a worker."""

    def __init__(self, engine, batch_window: float = 0.0):
        self.engine = engine
        self.batch_window = batch_window

    async def stream(self, prompt: str):
        from ..engine.grammar import single_command_schema
        from ..engine.llm_engine import GenRequest
        ch = Chan(4096)
        loop = asyncio.get_running_loop()
        tok = self.engine.tok

        def push(ids):                                  # engine thread
            loop.call_soon_threadsafe(ch.try_put, (tok.decode(ids), False))
        req = GenRequest(tok.encode_prompt(prompt), single_command_schema(), on_tokens=push)

        async def run():
            try:
                if self.batch_window:
                    await asyncio.sleep(self.batch_window)
                if hasattr(self.engine, "submit_batch") and getattr(self.engine, "is_gpu", False):
                    await asyncio.wrap_future(self.engine.submit_batch([req]))
                else:
                    await loop.run_in_executor(None, self.engine.generate, [req])
                await asyncio.sleep(0)          # the last call_soon_threadsafe pushes
                ch.try_put(("", True))
            except Exception as e:  # noqa: BLE001
                ch.try_put(e)
            finally:
                ch.close()
        task = loop.create_task(run())
        try:
            async for item in ch:
                if isinstance(item, Exception):
                    raise item
                yield item
        finally:
            if not task.done():
                await task


class StreamingCommandParser:
    def __init__(self, backend: StreamingBackend | None, fallback: CommandParser | None,
                 enabled: bool = True, *, max_buffer_time: float = 2.0,
                 max_tokens_per_phrase: int = 50):
        self.backend = backend
        self.fallback = fallback
        self.enabled = enabled and backend is not None
        self.max_buffer_time = max_buffer_time
        self.max_tokens_per_phrase = max_tokens_per_phrase

    async def parse_command_streaming(self, transcription: str) -> StreamingResult:
        if not self.enabled:
            if self.fallback is None:
                raise RuntimeError("streaming disabled and no fallback parser")
            return self._fallback_result(await self.fallback.parse_command(transcription))
        if transcription == "":
            return self._fallback_result(Command("unknown", {}, 0.0, "I didn't hear anything."))
        res = StreamingResult()
        res._task = asyncio.get_running_loop().create_task(self._produce(transcription, res))
        return res

    async def _produce(self, transcription: str, res: StreamingResult) -> None:
        m = res.metrics
        pb = PhraseBuffer(self.max_buffer_time, self.max_tokens_per_phrase)
        full: list[str] = []
        try:
            async for content, done in self.backend.stream(build_streaming_prompt(transcription)):
                if content:
                    if not m.first_token_time:
                        m.first_token_time = time.monotonic()
                    m.token_count += 1
                    await res.visual_tokens.put(content)
                    await res.token_stream.put(content)
                    full.append(content)
                    phrase = pb.add_token(content)
                    if phrase:
                        if not m.first_phrase_time:
                            m.first_phrase_time = time.monotonic()
                        m.phrase_count += 1
                        await res.audio_phrases.put(phrase)
                if done:
                    break
            rest = pb.flush()
            if rest:
                m.phrase_count += 1
                await res.audio_phrases.put(rest)
            m.completion_time = time.monotonic()
            try:
                cmd = parse_response("".join(full))
            except Exception as e:  # noqa: BLE001
                res.errors.try_put(ValueError(f"error parsing final command: {e}"))
                return
            await res.final_command.put(cmd)
            log.info("streaming command completed tokens=%d phrases=%d", m.token_count,
                     m.phrase_count)
        except asyncio.CancelledError:
            m.interrupt_count += 1
        except ChannelClosed:
            m.interrupt_count += 1
        except Exception as e:  # noqa: BLE001
            res.errors.try_put(ConnectionError(f"failed to create streaming request: {e}"))
        finally:
            res.close_outputs()

    def _fallback_result(self, cmd: Command) -> StreamingResult:
        return completed_result(cmd)


    async def test_streaming_connection(self, timeout: float = 10.0) -> None:
        if not self.enabled:
            raise RuntimeError("streaming is disabled, using fallback parser")
        res = await self.parse_command_streaming("hello")

        async def first():
            tok_task = asyncio.ensure_future(res.token_stream.get())
            err_task = asyncio.ensure_future(res.errors.get())
            done, pending = await asyncio.wait({tok_task, err_task},
                                               return_when=asyncio.FIRST_COMPLETED)
            for p in pending:
                p.cancel()
            d = done.pop()
            if d is err_task:
                raise RuntimeError(f"streaming test error: {d.result()}")
            try:
                d.result()
            except ChannelClosed:
                e, ok = res.errors.try_get()
                raise RuntimeError(f"streaming test error: {e if ok else 'no tokens'}") from None
        try:
            await asyncio.wait_for(first(), timeout)
        except asyncio.TimeoutError:
            raise RuntimeError("streaming test timeout") from None
        finally:
            res.cancel()


def completed_result(cmd: Command) -> StreamingResult:
    """A finished streaming result carrying one already-parsed command (the
    disabled-streaming fallback, :422-454, and the shared GPU decode that the
    bridge monitors instead of a second parse)."""
    res = StreamingResult()
    now = time.monotonic()
    for ch in (res.visual_tokens, res.audio_phrases, res.token_stream):
        ch.try_put(cmd.response)
    res.final_command.try_put(cmd)
    m = res.metrics
    m.first_token_time = m.first_phrase_time = m.completion_time = now
    m.token_count = m.phrase_count = 1
    res.close_outputs()
    return res
