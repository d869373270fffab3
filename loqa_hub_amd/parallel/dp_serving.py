"""Data-parallel serving over the GPUs of one node.

The hub front-end (gRPC relays, arbitration, HTTP, NATS) stays on the CPU in
one process; every GPU gets ONE worker process (spawned, pinned to
``cuda:<rank>``) that owns a full on-device pipeline (``GPUVoiceProcessor``:
batched Whisper -> constrained multi-command decode -> command queue / NATS).
Arbitration winners are routed to the least-loaded healthy worker
(``LeastLoadedRouter``: fewest queued utterances, ties -> lowest rank); each
worker micro-batches whatever it receives, so continuous batching happens per
GPU. The reference serialises every relay behind one global arbitration
window and one HTTP STT/Ollama service (``audio_service.go:89,435``); it has no
multi-GPU anything.

Failure handling (reference: none beyond service retries):

* crash  - a worker process that exits is detected by the monitor;
* hang   - every worker heartbeats (its own thread) with the age of its last
           completed utterance while it has work in flight: no progress for
           ``watchdog_s`` with work queued = a hung GPU;
* either way the router marks it unhealthy, the process is killed (exact PID,
  it is our child), and its queued utterances are re-dispatched to the
  surviving workers; with no survivor they complete with the STT-failed
  reply. ``FAULT_INJECT=gpu_kill:<rank>[@n]`` drives this path.

``metrics()`` aggregates per-worker counters (D3) for ``/api/metrics``.

PCM transport: each worker owns a ring of ``LOQA_DP_SHM_SLOTS`` 30 s slots in
POSIX shared memory, created by the front end. At dispatch the front end
copies the winner's PCM16 into a free slot of the chosen worker and sends only
(slot, length) over the request queue; the GPU worker has the whole ring
pinned (``hipHostRegister``) and its STT upload is one ``hipMemcpyAsync``
straight from the slot (``engine/pcm_staging.RegisteredPcm``). The slot goes
back to the front end's free list when the utterance's result arrives (or its
worker dies). Longer utterances, or a full ring, travel as bytes in the queue
item as before.
"""
from __future__ import annotations

import asyncio
import dataclasses
import itertools
import logging
import multiprocessing as mp
import os
import queue
import threading
import time

import numpy as np

from ..transport.audio_service import MSG_STT_FAILED, UtteranceResult
from .dp_router import LeastLoadedRouter

log = logging.getLogger("loqa.dp")

SHM_SLOTS = int(os.environ.get("LOQA_DP_SHM_SLOTS", "48"))
SHM_SLOT_BYTES = 480000 * 2          # one 30 s window of PCM16


def create_pcm_rings(n: int, slots: int, slot_bytes: int, shm_dir: str = "/dev/shm") -> list:
    """One shared-memory PCM ring per worker, every page reserved up front, or
    [] (inline pickled PCM) when the space is not there. A POSIX segment is a
    sparse file: without the reservation a tmpfs limit (a container's default
    64 MB /dev/shm) would surface as SIGBUS on the first touch past it - in the
    front end's event loop copying PCM in, or in a worker pinning the ring."""
    from multiprocessing import shared_memory
    size = slots * slot_bytes
    try:
        st = os.statvfs(shm_dir)
        free = st.f_bavail * st.f_frsize
    except OSError:
        free = None
    if free is not None and free < n * size + (16 << 20):
        log.warning("PCM rings need %.0f MB of %s, %.0f MB free: sending PCM inline",
                    n * size / 1e6, shm_dir, free / 1e6)
        return []
    made: list = []
    try:
        for _ in range(n):
            m = shared_memory.SharedMemory(create=True, size=size)
            made.append(m)
            fd = getattr(m, "_fd", -1)
            if fd >= 0 and hasattr(os, "posix_fallocate"):
                os.posix_fallocate(fd, 0, size)   # ENOSPC here, not SIGBUS later
    except OSError as e:
        log.warning("PCM ring allocation failed (%s): sending PCM inline", e)
        for m in made:
            try:
                m.close()
                m.unlink()
            except OSError:
                pass
        return []
    return made


class _WorkerPcmRing:
    """Worker side of its shared-memory PCM ring (mapped, and pinned on a GPU)."""

    def __init__(self, name: str, slot_bytes: int, device: str):
        from multiprocessing import shared_memory
        self.shm = shared_memory.SharedMemory(name=name)
        self.slot_bytes = slot_bytes
        import ctypes
        self.addr = ctypes.addressof(ctypes.c_char.from_buffer(self.shm.buf))
        self.registered = False
        if device.startswith("cuda"):
            from ..engine.pcm_staging import host_register
            self.registered = host_register(self.addr, self.shm.size)
            if not self.registered:
                log.warning("hipHostRegister of the PCM ring failed: staging copies instead")

    def samples(self, slot: int, nbytes: int):
        """(int16 view of the slot, a RegisteredPcm for the GPU upload or None)."""
        off = slot * self.slot_bytes
        view = np.frombuffer(self.shm.buf, dtype="<i2", count=nbytes // 2, offset=off)
        if not self.registered:
            return view, None
        from ..engine.pcm_staging import RegisteredPcm
        return view, RegisteredPcm(view, self.addr + off)

    def close(self) -> None:
        if self.registered:
            from ..engine.pcm_staging import host_unregister
            host_unregister(self.addr)
        try:
            self.shm.close()
        except BufferError:
            pass                      # a view is still referenced: the OS unmaps at exit


# --------------------------------------------------------------- worker side
async def _build_worker_processor(spec: dict, device: str):
    """The per-GPU composition - the same one ``server.build_gpu_processor``
    gives the 1-GPU hub, so every DP worker serves what the 1-GPU hub serves
    (the reference's winner path, ``audio_service.go:590-761``):

    * STT -> ONE constrained multi-command decode -> command queue publishing
      every command on ``loqa.voice.commands`` / ``loqa.devices.commands.*``
      (``audio_service.go:109-156``) over this worker's OWN NATS connection to
      the hub's broker (``spec["nats_url"]``);
    * the streaming-predictive bridge on that decode, over this worker's skill
      manager (the builtin skills + ``skills_dir``);
    * the reply voice (``HUB_TTS_BACKEND``: on-device VITS on this GPU),
      progressive phrase by phrase on NATS ``audio.<relay>`` when streaming is
      enabled (``audio_service.go:693-761``).

    ``spec["cfg"]`` is the hub's ``Config``."""
    from ..messaging.audio_stream_publisher import AudioStreamPublisher
    from ..messaging.nats_service import NATSService
    from ..server import build_gpu_processor, build_tts
    from ..skills import DefaultSkillLoader, SkillManager, SkillManagerConfig
    from ..skills.builtin.lights import LightsSkill
    cfg = spec["cfg"]
    skills = SkillManager(SkillManagerConfig(skills_dir=spec.get("skills_dir", "./skills"),
                                             config_store=spec.get("skills_config_store",
                                                                   "./data/skills")),
                          DefaultSkillLoader(skills_root=spec.get("skills_dir", "./skills")))
    await skills.register_plugin(LightsSkill())
    await skills.start()
    tts = build_tts(cfg, device)
    # engines first (minutes of warm-up for the large models), then the bus:
    # an idle connection is not left unanswered while the loop is blocked
    proc = build_gpu_processor(cfg, None, device, tts, skills=skills)
    nats = None
    if spec.get("nats_url"):
        nats = NATSService(spec["nats_url"], cfg.nats.reconnect_wait)
        try:
            await nats.connect()
        except Exception as e:  # noqa: BLE001 - as the hub: serve without the bus
            log.warning("worker cannot connect to NATS at %s: %s", spec["nats_url"], e)
    proc.pipeline.nats = nats
    if nats is not None and nats.conn is not None:
        proc.attach_publisher(AudioStreamPublisher(nats.conn))
    proc.dp_resources = (nats, skills)
    return proc


async def _close_worker_processor(proc) -> None:
    close = getattr(proc, "close", None)
    if close is not None:
        await close()
    nats, skills = getattr(proc, "dp_resources", (None, None))
    if skills is not None:
        await skills.stop()
    if nats is not None:
        await nats.close()


def _worker_main(rank: int, spec: dict, req_q, resp_q) -> None:
    """One GPU worker. Requests: ``("utt", rid, relay, request_id, pcm16 bytes,
    sample rate, transcript hint)`` - the relay's raw PCM16-LE bytes, handed
    to the processor as int16 samples (staged into a pinned slot by the STT
    engine, converted on the device: no host float round trip) - or
    ``("int", relay)``: interrupt the reply that relay is still receiving."""
    from ..utils.faults import set_faults
    spec = dict(spec, rank=rank)
    fi = set_faults(spec.get("fault_inject"))
    kill_after = fi.gpu_kill_after(rank)
    device = spec.get("device", "cuda")
    if device == "cuda":
        import torch
        device = f"cuda:{rank % max(1, torch.cuda.device_count())}"
    if device.startswith("cuda"):
        import torch
        torch.cuda.set_device(device)
    loop = asyncio.new_event_loop()
    asyncio.set_event_loop(loop)
    factory = spec.get("factory") or _build_worker_processor
    proc = factory(spec, device)
    if asyncio.iscoroutine(proc):
        proc = loop.run_until_complete(proc)
    takes_pcm16 = getattr(proc, "takes_pcm16", False)
    state = {"inflight": 0, "last_progress": time.monotonic(), "done": 0, "stop": False}
    lock = threading.Lock()

    def heartbeat() -> None:
        while not state["stop"]:
            with lock:
                age = time.monotonic() - state["last_progress"]
                st = dict(getattr(proc, "stats", {}))
                tts = getattr(proc, "tts", None)
                for k, v in (getattr(tts, "stats", None) or {}).items():
                    st["tts_" + k] = v
                hb = {"inflight": state["inflight"], "since_progress": age,
                      "done": state["done"], "stats": st}
            resp_q.put(("hb", rank, hb))
            time.sleep(spec.get("heartbeat_s", 0.5))

    ring = None
    if spec.get("pcm_shm"):
        ring = _WorkerPcmRing(spec["pcm_shm"][rank], spec["pcm_shm_slot_bytes"], device)

    async def handle(item) -> None:
        _, rid, relay_id, request_id, data, sr, hint = item
        reg = None
        if isinstance(data, tuple):               # ("shm", slot, nbytes)
            pcm16, reg = ring.samples(data[1], data[2])
        else:
            pcm16 = np.frombuffer(data, dtype="<i2")
        try:
            if takes_pcm16:
                kw = {"pcm16": pcm16}
                if reg is not None:
                    kw = {"pcm_slot": reg}
                if hint:
                    kw["transcript_hint"] = hint
                res = await proc.process(relay_id, request_id, np.zeros(0, np.float32), sr, **kw)
            else:
                res = await proc.process(relay_id, request_id,
                                         pcm16.astype(np.float32) / 32767.0, sr)
            out = dataclasses.asdict(res)
        except Exception as e:  # noqa: BLE001
            out = dataclasses.asdict(UtteranceResult(success=False, command="error",
                                                     response_text=MSG_STT_FAILED, error=str(e)))
        with lock:
            state["inflight"] -= 1
            state["done"] += 1
            state["last_progress"] = time.monotonic()
        resp_q.put(("res", rank, (rid, out)))

    def interrupt(relay_id: str) -> None:
        fn = getattr(proc, "interrupt_relay", None)
        if fn is not None:
            fn(relay_id)

    def reader() -> None:
        received = 0
        while True:
            item = req_q.get()
            if item is None:
                loop.call_soon_threadsafe(loop.stop)
                return
            if item[0] == "int":
                loop.call_soon_threadsafe(interrupt, item[1])
                continue
            received += 1
            if kill_after is not None and received >= kill_after:
                os._exit(17)  # injected GPU-worker crash (FAULT_INJECT=gpu_kill)
            with lock:
                if state["inflight"] == 0:
                    state["last_progress"] = time.monotonic()
                state["inflight"] += 1
            asyncio.run_coroutine_threadsafe(handle(item), loop)

    threading.Thread(target=heartbeat, daemon=True).start()
    threading.Thread(target=reader, daemon=True).start()
    resp_q.put(("ready", rank, None))
    try:
        loop.run_forever()
        loop.run_until_complete(_close_worker_processor(proc))
    finally:
        state["stop"] = True
        if ring is not None:
            ring.close()


# --------------------------------------------------------------- front side
@dataclasses.dataclass
class _Req:
    args: tuple
    fut: asyncio.Future
    worker: int = -1
    attempts: int = 0
    session: str = ""
    shm_slot: int = -1          # slot of the worker's PCM ring holding the samples


class _RemoteReply:
    """The front end's handle on a reply a worker is speaking (a streaming
    session's cancel target)."""

    def __init__(self, dp: "DPVoiceProcessor", relay_id: str):
        self.dp, self.relay_id = dp, relay_id

    def cancel(self) -> None:
        rid = self.dp._relay_req.get(self.relay_id)
        req = self.dp._reqs.get(rid) if rid is not None else None
        if req is not None and req.worker >= 0:
            self.dp._send_interrupt(req.worker, self.relay_id)


class DPVoiceProcessor:
    """``VoiceProcessor`` over one worker process per GPU."""

    takes_pcm16 = True      # AudioService hands over the relay's raw PCM16 samples
    tts = None              # the reply voice lives in the workers

    def __init__(self, spec: dict, n_workers: int, *, watchdog_s: float = 60.0,
                 ready_timeout: float = 900.0, max_attempts: int = 3):
        self.spec = dict(spec)
        cfg = self.spec.get("cfg")
        self.progressive = bool(cfg is not None and cfg.streaming.enabled
                                and cfg.gpu.tts_backend != "none")
        self.streaming = None
        self._relay_req: dict[str, int] = {}
        self.n = n_workers
        self.watchdog_s = watchdog_s
        self.ready_timeout = ready_timeout
        self.max_attempts = max_attempts
        self.router = LeastLoadedRouter(n_workers)
        self._ids = itertools.count()
        self._reqs: dict[int, _Req] = {}
        self._pending: list[set[int]] = [set() for _ in range(n_workers)]
        self._hb: list[dict] = [{} for _ in range(n_workers)]
        self._last_hb = [0.0] * n_workers
        self._ready = [False] * n_workers
        self.failures: list[dict] = []
        self._running = False
        self._served = 0
        self._shm: list = []
        self._shm_free: list[list[int]] = []
        self.pcm_shm_sent = 0
        self.pcm_inline_sent = 0

    # lifecycle
    async def start(self) -> None:
        ctx = mp.get_context("spawn")
        if SHM_SLOTS > 0 and "pcm_shm" not in self.spec:
            self._shm = create_pcm_rings(self.n, SHM_SLOTS, SHM_SLOT_BYTES)
            if self._shm:
                self._shm_free = [list(range(SHM_SLOTS)) for _ in range(self.n)]
                self.spec["pcm_shm"] = [m.name for m in self._shm]
                self.spec["pcm_shm_slot_bytes"] = SHM_SLOT_BYTES
        self._req_qs = [ctx.Queue() for _ in range(self.n)]
        self._resp_q = ctx.Queue()
        self._procs = [ctx.Process(target=_worker_main, args=(r, self.spec, self._req_qs[r],
                                                              self._resp_q), daemon=True)
                       for r in range(self.n)]
        for p in self._procs:
            p.start()
        self._loop = asyncio.get_running_loop()
        self._running = True
        self._reader = threading.Thread(target=self._read, daemon=True)
        self._reader.start()
        t0 = time.monotonic()
        while not all(self._ready[r] or not self._procs[r].is_alive() for r in range(self.n)):
            if time.monotonic() - t0 > self.ready_timeout:
                raise TimeoutError("DP workers did not become ready")
            await asyncio.sleep(0.05)
        for r in range(self.n):
            if not self._ready[r]:
                self._fail_worker(r, "died during start-up")
        now = time.monotonic()
        self._last_hb = [now] * self.n
        self._monitor = asyncio.ensure_future(self._watch())

    async def close(self) -> None:
        self._running = False
        if getattr(self, "_monitor", None):
            self._monitor.cancel()
        for r, p in enumerate(self._procs):
            if p.is_alive():
                self._req_qs[r].put(None)
        for p in self._procs:
            p.join(timeout=10)
            if p.is_alive():
                p.kill()
                p.join(timeout=5)
        for m in self._shm:
            try:
                m.close()
                m.unlink()
            except (FileNotFoundError, BufferError):
                pass
        self._shm = []

    # routing
    async def process(self, relay_id: str, request_id: str, audio: np.ndarray,
                      sample_rate: int, transcript_hint: str | None = None,
                      pcm16: np.ndarray | None = None, pcm_slot=None) -> UtteranceResult:
        """``pcm16``: the relay's raw samples as received (``AudioService``
        passes them: ``takes_pcm16``); they travel to the worker as PCM16-LE
        bytes. Float ``audio`` (other callers) is quantised once here."""
        if pcm16 is not None:
            data = np.ascontiguousarray(pcm16, dtype="<i2").tobytes()
        else:
            data = np.clip(np.round(np.asarray(audio, np.float32) * 32767.0), -32768,
                           32767).astype("<i2").tobytes()
        if pcm_slot is not None:          # never handed out (no new_pcm_slot here)
            pcm_slot.release()
        rid = next(self._ids)
        req = _Req(("utt", relay_id, request_id, data, sample_rate, transcript_hint),
                   self._loop.create_future())
        self._reqs[rid] = req
        self._relay_req[relay_id] = rid
        if self.streaming is not None and self.progressive:
            req.session = f"dp_{rid}_{request_id}"
            self.streaming.begin_speech_session(req.session, _RemoteReply(self, relay_id))
        self._dispatch(rid)
        try:
            return await req.fut
        finally:
            if self._relay_req.get(relay_id) == rid:
                del self._relay_req[relay_id]

    def attach_publisher(self, publisher) -> None:
        """Workers publish over their own NATS connections; the hub's
        publisher only delivers replies that were not already published."""

    def attach_streaming(self, components) -> None:
        self.streaming = components

    def interrupt_relay(self, relay_id: str, reason: str = "new_command") -> bool:
        """Forward a new-winner interrupt to the worker speaking to ``relay_id``."""
        rid = self._relay_req.get(relay_id)
        req = self._reqs.get(rid) if rid is not None else None
        if req is None or req.worker < 0:
            return False
        ih = self.streaming.interrupt_handler if self.streaming is not None else None
        if ih is not None and req.session in ih.active:
            ih.interrupt_session(req.session, reason)
        else:
            self._send_interrupt(req.worker, relay_id)
        return True

    def _send_interrupt(self, w: int, relay_id: str) -> None:
        if self.router.healthy[w]:
            self._req_qs[w].put(("int", relay_id))

    def _dispatch(self, rid: int) -> None:
        req = self._reqs[rid]
        req.attempts += 1
        try:
            w = self.router.pick()
        except RuntimeError:
            self._finish(rid, UtteranceResult(success=False, command="error",
                                              response_text=MSG_STT_FAILED,
                                              error="no healthy GPU workers"))
            return
        req.worker = w
        self._pending[w].add(rid)
        args = req.args[1:]
        data = args[2]
        if self._shm and len(data) <= SHM_SLOT_BYTES and self._shm_free[w]:
            slot = self._shm_free[w].pop()
            off = slot * SHM_SLOT_BYTES
            self._shm[w].buf[off:off + len(data)] = data
            req.shm_slot = slot
            args = args[:2] + (("shm", slot, len(data)),) + args[3:]
            self.pcm_shm_sent += 1
        else:
            self.pcm_inline_sent += 1
        self._req_qs[w].put(("utt", rid) + args)

    def _free_shm(self, req: _Req) -> None:
        if req.shm_slot >= 0 and req.worker >= 0 and self._shm:
            self._shm_free[req.worker].append(req.shm_slot)
        req.shm_slot = -1

    def _finish(self, rid: int, res: UtteranceResult) -> None:
        req = self._reqs.pop(rid, None)
        if req is not None:
            self._free_shm(req)
        if req is not None and req.session and self.streaming is not None:
            sm = (res.metrics or {}).get("speech", {}).get("streaming")
            self.streaming.end_speech_session(req.session, sm)
        if req is not None and not req.fut.done():
            req.fut.set_result(res)

    # worker -> front messages (reader thread -> event loop)
    def _read(self) -> None:
        while self._running:
            try:
                msg = self._resp_q.get(timeout=0.2)
            except queue.Empty:
                continue
            except (EOFError, OSError):
                return
            self._loop.call_soon_threadsafe(self._on_msg, msg)

    def _on_msg(self, msg) -> None:
        kind, w, payload = msg
        if kind == "ready":
            self._ready[w] = True
            self._last_hb[w] = time.monotonic()
        elif kind == "hb":
            self._hb[w] = payload
            self._last_hb[w] = time.monotonic()
        elif kind == "res":
            rid, d = payload
            if rid in self._pending[w]:
                self._pending[w].discard(rid)
                self.router.done(w)
            self._finish(rid, UtteranceResult(**d))
            self._served += 1

    # health
    async def _watch(self) -> None:
        period = max(0.05, self.spec.get("heartbeat_s", 0.5))
        while self._running:
            await asyncio.sleep(period)
            now = time.monotonic()
            for w in range(self.n):
                if not self.router.healthy[w]:
                    continue
                p = self._procs[w]
                hb = self._hb[w]
                if not p.is_alive():
                    self._fail_worker(w, f"process exited (code {p.exitcode})")
                elif now - self._last_hb[w] > self.watchdog_s:
                    self._fail_worker(w, "heartbeat lost")
                elif self._pending[w] and hb.get("inflight", 0) > 0 and \
                        hb.get("since_progress", 0.0) > self.watchdog_s:
                    self._fail_worker(w, "no progress (GPU hang)")

    def _fail_worker(self, w: int, why: str) -> None:
        if not self.router.healthy[w] and not self._pending[w]:
            return
        log.error("GPU worker %d unhealthy: %s; re-routing %d utterances", w, why,
                  len(self._pending[w]))
        self.failures.append({"worker": w, "reason": why, "rerouted": len(self._pending[w]),
                              "t": time.time()})
        self.router.mark_unhealthy(w)
        p = self._procs[w]
        if p.is_alive():
            p.kill()
        orphans, self._pending[w] = self._pending[w], set()
        for rid in sorted(orphans):
            req = self._reqs.get(rid)
            if req is None:
                continue
            self._free_shm(req)         # the dead worker's slot: its reader is gone
            if req.attempts >= self.max_attempts:
                self._finish(rid, UtteranceResult(success=False, command="error",
                                                  response_text=MSG_STT_FAILED,
                                                  error=f"worker failures: {why}"))
            else:
                self._dispatch(rid)

    @property
    def stats(self) -> dict:
        """The workers' processor counters summed (as of their last heartbeat)."""
        out: dict = {}
        for hb in self._hb:
            for k, v in (hb.get("stats") or {}).items():
                if isinstance(v, (int, float)) and not isinstance(v, bool):
                    out[k] = out.get(k, 0) + v
        out["served"] = self._served
        out["pcm_shm_sent"] = self.pcm_shm_sent
        out["pcm_inline_sent"] = self.pcm_inline_sent
        return out

    def metrics(self) -> dict:
        """Per-worker counters aggregated on the front-end (D3)."""
        workers = []
        for w in range(self.n):
            hb = self._hb[w]
            workers.append({"rank": w, "healthy": self.router.healthy[w],
                            "queued": len(self._pending[w]), "done": hb.get("done", 0),
                            "stats": hb.get("stats", {})})
        return {"workers": workers, "healthy": sum(self.router.healthy),
                "utterances": sum(x["done"] for x in workers), "failures": list(self.failures)}
