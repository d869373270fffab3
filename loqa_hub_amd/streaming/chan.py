"""Closable bounded async channel (the Go ``chan`` idiom on asyncio).

``put`` blocks when full, ``get`` raises ``ChannelClosed`` once the channel is
closed *and* drained; ``async for`` iterates until then. ``try_put`` is the
non-blocking ``select { case ch <- v: default: }``.
"""
from __future__ import annotations

import asyncio
from collections import deque


class ChannelClosed(Exception):
    pass


class Chan:
    def __init__(self, cap: int = 0):
        self.cap = max(1, cap)
        self._q: deque = deque()
        self._closed = False
        self._readable = asyncio.Event()
        self._writable = asyncio.Event()
        self._writable.set()

    def __len__(self) -> int:
        return len(self._q)

    @property
    def closed(self) -> bool:
        return self._closed

    def _update(self) -> None:
        if self._q or self._closed:
            self._readable.set()
        else:
            self._readable.clear()
        if len(self._q) < self.cap or self._closed:
            self._writable.set()
        else:
            self._writable.clear()

    async def put(self, v) -> None:
        while True:
            if self._closed:
                raise ChannelClosed("send on closed channel")
            if len(self._q) < self.cap:
                self._q.append(v)
                self._update()
                return
            await self._writable.wait()

    def try_put(self, v) -> bool:
        if self._closed or len(self._q) >= self.cap:
            return False
        self._q.append(v)
        self._update()
        return True

    async def get(self):
        while True:
            if self._q:
                v = self._q.popleft()
                self._update()
                return v
            if self._closed:
                raise ChannelClosed()
            await self._readable.wait()

    def try_get(self):
        """(value, True) or (None, False) without blocking."""
        if self._q:
            v = self._q.popleft()
            self._update()
            return v, True
        return None, False

    def close(self) -> None:
        self._closed = True
        self._update()

    def __aiter__(self):
        return self

    async def __anext__(self):
        try:
            return await self.get()
        except ChannelClosed:
            raise StopAsyncIteration from None
