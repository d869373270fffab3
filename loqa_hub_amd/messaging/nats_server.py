"""Embedded NATS-protocol broker (asyncio).

Lets the hub run self-contained (and the tests run without a NATS server,
replacing the reference CI's NATS 2.10 service container, ``ci.yml:21-40``),
while staying wire-compatible: relays, skills and devices that speak real NATS
can connect to it. Supports PUB/SUB/UNSUB/PING/PONG, queue groups and the
``*`` / ``>`` subject wildcards.
"""
from __future__ import annotations

import asyncio
import json
import logging
import random

log = logging.getLogger("loqa.nats.server")


def subject_matches(pattern: str, subject: str) -> bool:
    p, s = pattern.split("."), subject.split(".")
    for i, tok in enumerate(p):
        if tok == ">":
            return len(s) > i
        if i >= len(s) or (tok != "*" and tok != s[i]):
            return False
    return len(p) == len(s)


class _Client:
    def __init__(self, cid: int, w: asyncio.StreamWriter):
        self.cid, self.w = cid, w
        self.subs: dict[str, tuple[str, str | None]] = {}
        self.name = ""


class NATSServer:
    def __init__(self, host: str = "127.0.0.1", port: int = 0):
        self.host, self.port = host, port
        self._server: asyncio.AbstractServer | None = None
        self._clients: dict[int, _Client] = {}
        self._next = 0
        self.msgs_routed = 0

    @property
    def url(self) -> str:
        return f"nats://{self.host}:{self.port}"

    async def start(self) -> "NATSServer":
        self._server = await asyncio.start_server(self._handle, self.host, self.port)
        self.port = self._server.sockets[0].getsockname()[1]
        return self

    async def stop(self) -> None:
        if self._server:
            self._server.close()
            for c in list(self._clients.values()):
                c.w.close()
            await self._server.wait_closed()

    async def _handle(self, r: asyncio.StreamReader, w: asyncio.StreamWriter) -> None:
        self._next += 1
        c = _Client(self._next, w)
        self._clients[c.cid] = c
        info = {"server_id": "loqa-embedded", "server_name": "loqa-embedded", "version": "2.10.0",
                "proto": 1, "host": self.host, "port": self.port, "headers": False,
                "max_payload": 8 * 1024 * 1024, "client_id": c.cid}
        w.write(b"INFO " + json.dumps(info).encode() + b"\r\n")
        try:
            while True:
                line = await r.readline()
                if not line:
                    break
                op = line.split(b" ", 1)[0].strip().upper()
                if op == b"PUB":
                    parts = line.split()
                    subj = parts[1].decode()
                    reply = parts[2].decode() if len(parts) == 4 else None
                    n = int(parts[-1])
                    payload = (await r.readexactly(n + 2))[:n]
                    self._route(subj, reply, payload)
                elif op == b"SUB":
                    parts = line.split()
                    subj = parts[1].decode()
                    queue = parts[2].decode() if len(parts) == 4 else None
                    c.subs[parts[-1].decode()] = (subj, queue)
                elif op == b"UNSUB":
                    parts = line.split()
                    c.subs.pop(parts[1].decode(), None)
                elif op == b"PING":
                    w.write(b"PONG\r\n")
                elif op == b"CONNECT":
                    try:
                        c.name = json.loads(line[8:]).get("name", "")
                    except ValueError:
                        pass
                elif op in (b"PONG", b""):
                    pass
                else:
                    w.write(b"-ERR 'Unknown Protocol Operation'\r\n")
                await w.drain()
        except (ConnectionError, asyncio.IncompleteReadError):
            pass
        finally:
            self._clients.pop(c.cid, None)
            try:
                w.close()
            except Exception:
                pass

    def _route(self, subj: str, reply: str | None, payload: bytes) -> None:
        groups: dict[str, list[tuple[_Client, str]]] = {}
        for c in list(self._clients.values()):
            for sid, (pat, queue) in c.subs.items():
                if subject_matches(pat, subj):
                    if queue:
                        groups.setdefault(queue, []).append((c, sid))
                    else:
                        self._deliver(c, sid, subj, reply, payload)
        for members in groups.values():
            c, sid = random.choice(members)
            self._deliver(c, sid, subj, reply, payload)

    def _deliver(self, c: _Client, sid: str, subj: str, reply: str | None, payload: bytes) -> None:
        hdr = (f"MSG {subj} {sid} {reply} {len(payload)}\r\n" if reply
               else f"MSG {subj} {sid} {len(payload)}\r\n")
        try:
            c.w.write(hdr.encode() + payload + b"\r\n")
            self.msgs_routed += 1
        except Exception:
            pass


def main(argv=None) -> int:
    """Stand-alone broker process: ``python -m loqa_hub_amd.messaging.nats_server
    [--port P]`` prints ``port <n>`` once listening and exits when its stdin
    closes (so it never outlives the process that started it)."""
    import argparse
    import sys
    import threading
    ap = argparse.ArgumentParser()
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=0)
    args = ap.parse_args(argv)
    loop = asyncio.new_event_loop()
    srv = loop.run_until_complete(NATSServer(args.host, args.port).start())
    print(f"port {srv.port}", flush=True)

    def watch_stdin():
        sys.stdin.read()                      # EOF: the parent is gone
        loop.call_soon_threadsafe(loop.stop)

    threading.Thread(target=watch_stdin, daemon=True).start()
    loop.run_forever()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
