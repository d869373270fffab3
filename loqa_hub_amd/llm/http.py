"""HTTP client seam for the external-service backends (config 1 / fallback).

Mirrors the reference's ``HTTPClient`` DI interface (``mock_interfaces.go:31-33``)
so parsers and service clients are testable without a network:
``AiohttpClient`` is the real client, ``MockHTTPClient`` (``mock_interfaces.go:36-75``)
answers from canned responses.
"""
from __future__ import annotations

import json
from dataclasses import dataclass, field
from typing import AsyncIterator, Protocol


@dataclass
class HTTPResponse:
    status: int
    body: bytes = b""
    headers: dict = field(default_factory=dict)

    def json(self):
        return json.loads(self.body)


class HTTPClient(Protocol):
    async def request(self, method: str, url: str, *, body: bytes | None = None,
                      headers: dict | None = None, timeout: float = 30.0) -> HTTPResponse: ...

    def stream_lines(self, method: str, url: str, *, body: bytes | None = None,
                     headers: dict | None = None, timeout: float = 30.0) -> AsyncIterator[bytes]: ...


class AiohttpClient:
    def __init__(self):
        self._session = None

    async def _s(self):
        import aiohttp
        if self._session is None or self._session.closed:
            self._session = aiohttp.ClientSession()
        return self._session

    async def request(self, method, url, *, body=None, headers=None, timeout=30.0) -> HTTPResponse:
        import aiohttp
        s = await self._s()
        async with s.request(method, url, data=body, headers=headers or {},
                             timeout=aiohttp.ClientTimeout(total=timeout)) as r:
            return HTTPResponse(r.status, await r.read(), dict(r.headers))

    async def stream_lines(self, method, url, *, body=None, headers=None, timeout=30.0):
        import aiohttp
        s = await self._s()
        async with s.request(method, url, data=body, headers=headers or {},
                             timeout=aiohttp.ClientTimeout(total=timeout)) as r:
            if r.status != 200:
                raise HTTPStatusError(r.status, await r.read())
            async for line in r.content:
                yield line

    async def close(self) -> None:
        if self._session is not None:
            await self._session.close()


class HTTPStatusError(Exception):
    def __init__(self, status: int, body: bytes = b""):
        super().__init__(f"HTTP status {status}: {body[:200]!r}")
        self.status, self.body = status, body


class MockHTTPClient:
    """Canned responses keyed by URL substring; records every request."""

    def __init__(self, responses: dict[str, HTTPResponse | Exception] | None = None,
                 default: HTTPResponse | None = None):
        self.responses = responses or {}
        self.default = default
        self.requests: list[tuple[str, str, bytes | None]] = []

    def _match(self, url: str):
        for k, v in self.responses.items():
            if k in url:
                return v
        return self.default

    async def request(self, method, url, *, body=None, headers=None, timeout=30.0) -> HTTPResponse:
        self.requests.append((method, url, body))
        r = self._match(url)
        if callable(r):
            r = r(body)
        if isinstance(r, Exception):
            raise r
        if r is None:
            raise ConnectionError(f"no mock response for {url}")
        return r

    async def stream_lines(self, method, url, *, body=None, headers=None, timeout=30.0):
        self.requests.append((method, url, body))
        r = self._match(url)
        if callable(r):
            r = r(body)
        if isinstance(r, Exception):
            raise r
        if r is None:
            raise ConnectionError(f"no mock response for {url}")
        if r.status != 200:
            raise HTTPStatusError(r.status, r.body)
        for line in r.body.splitlines(keepends=True):
            yield line


def create_mock_ollama(response_text, status: int = 200) -> MockHTTPClient:
    """``CreateMockHTTPClient`` equivalent: every /api/generate returns
    ``{"response": response_text, "done": true}``. ``response_text`` may be a
    callable ``prompt -> str`` to answer per request."""
    def gen(body):
        text = response_text(json.loads(body)["prompt"]) if callable(response_text) else response_text
        return HTTPResponse(status, json.dumps({"response": text, "done": True}).encode())
    return MockHTTPClient({"/api/generate": gen,
                           "/api/tags": HTTPResponse(200, b'{"models": []}')})
