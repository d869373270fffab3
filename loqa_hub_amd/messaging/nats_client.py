"""Minimal asyncio NATS client speaking the NATS text protocol
(INFO / CONNECT / PUB / SUB / UNSUB / MSG / PING / PONG / +OK / -ERR).

``nats-py`` is not available in this image; this client covers what the hub
uses from ``nats.go`` in the reference (``nats_service.go:88-115``): a named
connection, publish, subscribe with callbacks, infinite reconnect with a fixed
wait, disconnect/reconnect/closed callbacks, and statistics.
"""
from __future__ import annotations

import asyncio
import json
import logging
from dataclasses import dataclass
from typing import Awaitable, Callable
from urllib.parse import urlparse

log = logging.getLogger("loqa.nats")

Handler = Callable[["Msg"], Awaitable[None] | None]


@dataclass
class Msg:
    subject: str
    data: bytes
    reply: str | None = None
    sid: int = 0


@dataclass
class Statistics:
    in_msgs: int = 0
    out_msgs: int = 0
    in_bytes: int = 0
    out_bytes: int = 0
    reconnects: int = 0


class NATSError(Exception):
    pass


class NATSClient:
    def __init__(self, *, name: str = "loqa-hub", reconnect_wait: float = 2.0,
                 max_reconnects: int = -1, on_disconnect=None, on_reconnect=None, on_closed=None):
        self.name = name
        self.reconnect_wait = reconnect_wait
        self.max_reconnects = max_reconnects
        self.on_disconnect, self.on_reconnect, self.on_closed = on_disconnect, on_reconnect, on_closed
        self._r: asyncio.StreamReader | None = None
        self._w: asyncio.StreamWriter | None = None
        self._subs: dict[int, tuple[str, str | None, Handler]] = {}
        self._sid = 0
        self._reader_task: asyncio.Task | None = None
        self._pongs: list[asyncio.Future] = []
        self._closed = False
        self._connected = asyncio.Event()
        self.stats = Statistics()
        self.url = ""
        self.server_info: dict = {}

    # ------------------------------------------------------------- connection
    async def connect(self, url: str = "nats://localhost:4222", timeout: float = 2.0) -> None:
        self.url = url
        await asyncio.wait_for(self._open(), timeout)
        self._reader_task = asyncio.get_running_loop().create_task(self._read_loop())

    async def _open(self) -> None:
        u = urlparse(self.url if "://" in self.url else "nats://" + self.url)
        host, port = u.hostname or "localhost", u.port or 4222
        self._r, self._w = await asyncio.open_connection(host, port)
        line = await self._r.readline()
        if not line.startswith(b"INFO"):
            raise NATSError(f"unexpected greeting {line!r}")
        self.server_info = json.loads(line[5:].strip() or b"{}")
        opts = {"verbose": False, "pedantic": False, "name": self.name, "lang": "python",
                "version": "0.1.0", "protocol": 1, "headers": False}
        if u.username:
            opts.update({"user": u.username, "pass": u.password or ""})
        self._w.write(b"CONNECT " + json.dumps(opts).encode() + b"\r\nPING\r\n")
        await self._w.drain()
        while True:
            line = await self._r.readline()
            if not line:
                raise NATSError("connection closed during handshake")
            if line.startswith(b"PONG"):
                break
            if line.startswith(b"-ERR"):
                raise NATSError(line.decode().strip())
        for sid, (subj, queue, _) in self._subs.items():
            self._w.write(self._sub_line(subj, queue, sid))
        await self._w.drain()
        self._connected.set()

    @staticmethod
    def _sub_line(subj: str, queue: str | None, sid: int) -> bytes:
        return (f"SUB {subj} {queue} {sid}\r\n" if queue else f"SUB {subj} {sid}\r\n").encode()

    def is_connected(self) -> bool:
        return self._connected.is_set() and not self._closed

    async def _read_loop(self) -> None:
        while not self._closed:
            try:
                await self._read_messages()
            except (ConnectionError, asyncio.IncompleteReadError, OSError) as e:
                log.warning("NATS read error: %s", e)
            if self._closed:
                break
            self._connected.clear()
            if self.on_disconnect:
                self.on_disconnect(self)
            attempts = 0
            while not self._closed:
                if 0 <= self.max_reconnects <= attempts:
                    await self.close()
                    return
                attempts += 1
                await asyncio.sleep(self.reconnect_wait)
                try:
                    await self._open()
                    self.stats.reconnects += 1
                    if self.on_reconnect:
                        self.on_reconnect(self)
                    break
                except (OSError, NATSError, asyncio.IncompleteReadError):
                    continue

    async def _read_messages(self) -> None:
        r = self._r
        while True:
            line = await r.readline()
            if not line:
                raise ConnectionError("server closed connection")
            if line.startswith(b"MSG"):
                parts = line.split()
                subj, sid = parts[1].decode(), int(parts[2])
                reply = parts[3].decode() if len(parts) == 5 else None
                n = int(parts[-1])
                payload = await r.readexactly(n + 2)
                data = payload[:n]
                self.stats.in_msgs += 1
                self.stats.in_bytes += n
                sub = self._subs.get(sid)
                if sub:
                    try:
                        res = sub[2](Msg(subj, data, reply, sid))
                        if asyncio.iscoroutine(res):
                            asyncio.get_running_loop().create_task(res)
                    except Exception:  # subscriber errors never kill the reader
                        log.exception("NATS handler failed")
            elif line.startswith(b"PING"):
                self._w.write(b"PONG\r\n")
            elif line.startswith(b"PONG"):
                if self._pongs:
                    f = self._pongs.pop(0)
                    if not f.done():
                        f.set_result(True)
            elif line.startswith(b"-ERR"):
                log.warning("NATS server error: %s", line.decode().strip())
            # +OK / INFO ignored

    # --------------------------------------------------------------- messaging
    def publish_nowait(self, subject: str, data: bytes, reply: str | None = None) -> None:
        if not self.is_connected():
            raise NATSError("NATS connection not established")
        hdr = f"PUB {subject} {reply} {len(data)}\r\n" if reply else f"PUB {subject} {len(data)}\r\n"
        self._w.write(hdr.encode() + data + b"\r\n")
        self.stats.out_msgs += 1
        self.stats.out_bytes += len(data)

    async def publish(self, subject: str, data: bytes, reply: str | None = None) -> None:
        self.publish_nowait(subject, data, reply)
        await self._w.drain()

    async def flush(self, timeout: float = 2.0) -> None:
        fut = asyncio.get_running_loop().create_future()
        self._pongs.append(fut)
        self._w.write(b"PING\r\n")
        await self._w.drain()
        await asyncio.wait_for(fut, timeout)

    async def subscribe(self, subject: str, cb: Handler, queue: str | None = None) -> int:
        self._sid += 1
        sid = self._sid
        self._subs[sid] = (subject, queue, cb)
        if self.is_connected():
            self._w.write(self._sub_line(subject, queue, sid))
            await self._w.drain()
        return sid

    async def unsubscribe(self, sid: int) -> None:
        if self._subs.pop(sid, None) is not None and self.is_connected():
            self._w.write(f"UNSUB {sid}\r\n".encode())
            await self._w.drain()

    async def close(self) -> None:
        if self._closed:
            return
        self._closed = True
        self._connected.clear()
        if self._w is not None:
            try:
                self._w.close()
            except Exception:
                pass
        if self._reader_task is not None and self._reader_task is not asyncio.current_task():
            self._reader_task.cancel()
        if self.on_closed:
            self.on_closed(self)
