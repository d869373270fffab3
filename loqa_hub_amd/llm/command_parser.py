"""LLM intent parser with multi-command support (``internal/llm/command_parser.go``).

Two interchangeable backends behind one ``LLMBackend`` interface:

* ``GPUBackend``   - the on-device grammar-constrained decode (engine/llm_engine.py):
                     the default, one decode per utterance, JSON valid by construction;
* ``OllamaBackend``- ``POST {url}/api/generate`` with ``stream:false``
                     (command_parser.go:223-266), the reference's path, kept for
                     BASELINE config 1 (CPU Ollama, no GPU) and as a fallback.

``CommandParser`` keeps the reference's observable behaviour: compound detection,
multi-command prompt with fallback to a single-command parse on any error
(:339-376), the default responses, and ``parse_command`` returning a combined
command for multi-utterances (:104-121, :476-516).
"""
from __future__ import annotations

import asyncio
import json
import logging
from typing import Protocol

from .commands import (Command, MultiCommand, ParseError, create_combined_command,
                       detect_compound_utterance, parse_multi_command_response, parse_response,
                       split_compound_utterance)
from .http import AiohttpClient, HTTPClient
from .prompts import DEFAULT_UNCLEAR_RESPONSE, build_multi_command_prompt, build_prompt

log = logging.getLogger("loqa.parser")


class LLMBackend(Protocol):
    async def generate(self, prompt: str, *, kind: str, n_commands: int) -> str: ...

    async def test_connection(self) -> None: ...


class OllamaBackend:
    def __init__(self, url: str = "http://localhost:11434", model: str = "llama3.2:3b",
                 client: HTTPClient | None = None, timeout: float = 30.0):
        self.url, self.model = url.rstrip("/"), model
        self.client = client or AiohttpClient()
        self.timeout = timeout

    async def generate(self, prompt: str, *, kind: str = "single", n_commands: int = 1) -> str:
        body = json.dumps({"model": self.model, "prompt": prompt, "stream": False}).encode()
        try:
            r = await self.client.request("POST", self.url + "/api/generate", body=body,
                                          headers={"Content-Type": "application/json"},
                                          timeout=self.timeout)
        except Exception as e:
            raise ConnectionError(f"error making request to Ollama: {e}") from e
        if r.status != 200:
            raise ConnectionError(f"ollama API returned status {r.status}")
        try:
            return str(json.loads(r.body).get("response", ""))
        except ValueError as e:
            raise ValueError(f"error unmarshaling response: {e}") from e

    async def test_connection(self) -> None:
        r = await self.client.request("GET", self.url + "/api/tags", timeout=10)
        if r.status != 200:
            raise ConnectionError(f"ollama API returned status {r.status}")
        await self.generate("Respond with just 'OK'")


class GPUBackend:
    """Grammar-constrained decode on the local GPU engine. Requests from
    concurrent callers are micro-batched into one engine call."""

    def __init__(self, engine, *, min_response_tokens: int = 0, batch_window: float = 0.002):
        self.engine = engine
        self.min_response_tokens = min_response_tokens
        self.batch_window = batch_window
        self._pending: list[tuple[str, str, int, asyncio.Future]] = []
        self._flusher: asyncio.Task | None = None
        self._lock = None

    async def generate(self, prompt: str, *, kind: str = "single", n_commands: int = 1) -> str:
        loop = asyncio.get_running_loop()
        fut = loop.create_future()
        self._pending.append((prompt, kind, n_commands, fut))
        if self._flusher is None or self._flusher.done():
            self._flusher = loop.create_task(self._flush())
        return await fut

    async def _flush(self) -> None:
        await asyncio.sleep(self.batch_window)
        batch, self._pending = self._pending, []
        if not batch:
            return
        from ..engine.grammar import multi_command_schema, single_command_schema
        from ..engine.llm_engine import GenRequest
        tok = self.engine.tok
        reqs = []
        for prompt, kind, n, _ in batch:
            schema = (multi_command_schema(max(1, n), min_response_tokens=self.min_response_tokens)
                      if kind == "multi" else single_command_schema())
            reqs.append(GenRequest(tok.encode_prompt(prompt), schema))
        try:
            await asyncio.get_running_loop().run_in_executor(None, self.engine.generate, reqs)
        except Exception as e:
            for *_, f in batch:
                if not f.done():
                    f.set_exception(e)
            return
        for (_, _, _, f), r in zip(batch, reqs):
            if not f.done():
                f.set_result(r.output)

    async def test_connection(self) -> None:
        return None


class CommandParser:
    def __init__(self, backend: LLMBackend):
        self.backend = backend

    async def parse_command(self, transcription: str) -> Command:
        try:
            mc = await self.parse_multi_command(transcription)
        except Exception:
            return await self._parse_single(transcription)
        if not mc.is_multi or len(mc.commands) == 1:
            if mc.commands:
                return mc.commands[0]
            return await self._parse_single(transcription)
        return create_combined_command(mc)

    async def parse_multi_command(self, transcription: str) -> MultiCommand:
        if transcription == "":
            return MultiCommand([], False, transcription, "I didn't hear anything.")
        if not detect_compound_utterance(transcription):
            cmd = await self._parse_single(transcription)
            return MultiCommand([cmd], False, transcription, cmd.response)
        return await self._parse_compound(transcription)

    async def _parse_single(self, transcription: str) -> Command:
        if transcription == "":
            return Command("unknown", {}, 0.0, "I didn't hear anything.")
        try:
            raw = await self.backend.generate(build_prompt(transcription), kind="single", n_commands=1)
        except Exception as e:
            log.warning("error querying LLM: %s", e)
            return Command("unknown", {}, 0.0, "I'm having trouble understanding you right now.")
        try:
            cmd = parse_response(raw)
        except ParseError as e:
            log.warning("error parsing LLM response: %s", e)
            return Command("unknown", {}, 0.0, DEFAULT_UNCLEAR_RESPONSE)
        return cmd

    async def _parse_compound(self, transcription: str) -> MultiCommand:
        n = max(1, len(split_compound_utterance(transcription)))
        try:
            raw = await self.backend.generate(build_multi_command_prompt(transcription), kind="multi",
                                              n_commands=n)
            return parse_multi_command_response(raw, transcription)
        except Exception as e:
            log.warning("multi-command parse failed (%s); falling back to single parse", e)
            cmd = await self._parse_single(transcription)
            return MultiCommand([cmd], False, transcription, cmd.response)

    async def test_connection(self) -> None:
        await self.backend.test_connection()
