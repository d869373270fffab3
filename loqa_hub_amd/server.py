"""Hub composition root (``internal/server/server.go``).

Builds: SQLite database -> voice-events store -> HTTP API; NATS service (and
the embedded broker when ``NATS_URL`` is ``embedded``); skill manager with the
builtin skills plus ``./skills`` auto-load; the voice processor (GPU pipeline
or external services) behind the gRPC ``AudioService``; streaming components
when enabled. Serves HTTP (``/health`` -> ``ok\\n`` (:137-142),
``/api/voice-events[/…]``, ``/api/skills[/…]``, ``/api/streaming/*``,
``/api/metrics``) and gRPC ``audio.AudioService/StreamAudio`` on
``cfg.server.grpc_port`` (:98-125). Deliberate differences from the reference:
the skills and streaming APIs are routed (the reference leaves them unrouted,
SURVEY C11), and every service reads the one config object.

GPU engines are built lazily by ``build_gpu_processor`` so a CPU-only hub
(config 1) never imports the HIP path.
"""
from __future__ import annotations

import os

import asyncio
import logging

from aiohttp import web

from .api.metrics import MetricsHandler
from .api.skills import SkillsHandler
from .api.streaming import StreamingHandler
from .api.voice_events import VoiceEventsHandler
from .config import Config
from .messaging.audio_stream_publisher import AudioStreamPublisher
from .messaging.nats_service import NATSService
from .skills import DefaultSkillLoader, SkillManager, SkillManagerConfig
from .skills.builtin.lights import LightsSkill
from .storage.database import Database
from .storage.voice_events_store import VoiceEventsStore
from .transport.audio_service import AudioService

log = logging.getLogger("loqa.server")


def build_tts(cfg: Config, device: str = "cuda:0"):
    """The reply voice (``audio_service.go:180-195``) from ``HUB_TTS_BACKEND``:
    ``gpu`` -> on-device VITS (``HUB_TTS_CHECKPOINT``, else the random-init
    ``HUB_TTS_MODEL``) on the serving GPU,
    ``http`` / ``openai`` -> the OpenAI-compatible client (``TTS_URL``; its
    connection is tested in ``HubServer.start`` with the reference's
    fallback rule), ``none`` -> text-only replies."""
    b = cfg.gpu.tts_backend
    if b == "none":
        return None
    if b == "gpu":
        from .engine.tts_engine import VitsTTSEngine
        from .models.configs import vits_config
        # phrases arriving within this window share one synthesis (a VITS call
        # at 1-2 phrases is launch / latency bound)
        win = float(os.environ.get("LOQA_TTS_BATCH_WINDOW_MS", "3")) / 1e3
        ckpt = cfg.gpu.tts_checkpoint or None
        return VitsTTSEngine(None if ckpt else vits_config(cfg.gpu.tts_model), device,
                             seed=cfg.gpu.seed, batch_window=win, checkpoint=ckpt,
                             format_policy=cfg.gpu.tts_format_policy)
    if b in ("http", "openai"):
        from .llm.tts import OpenAITTSClient
        return OpenAITTSClient(cfg.tts)
    raise ValueError(f"unknown HUB_TTS_BACKEND {b!r} (gpu | http | none)")


def build_bridge(skills_manager=None, tts=None, fallback_parser=None):
    """The streaming-predictive bridge and its stack (``audio_service.go:345-405``):
    classifier + reliability tracker, predictive engine and async execution
    pipeline over the skill manager (the hub's skills, the reference's
    always-failing adapter when there are none), status manager speaking
    through ``tts``. On the GPU path the classification and the streaming
    result both come from the one constrained decode, so ``fallback_parser``
    only serves callers without a parse."""
    from .predictive.async_execution import AsyncExecutionPipeline
    from .predictive.bridge import StreamingPredictiveBridge
    from .predictive.classifier import CommandClassifier
    from .predictive.engine import PredictiveResponseEngine
    from .predictive.reliability import DeviceReliabilityTracker
    from .predictive.skill_adapter import NullSkillManager, SkillManagerAdapter
    from .predictive.status_manager import StatusManager
    from .streaming.parser import StreamingCommandParser
    adapter = SkillManagerAdapter(skills_manager) if skills_manager is not None else NullSkillManager()
    rel = DeviceReliabilityTracker()
    clf = CommandClassifier(fallback_parser, rel)
    engine = PredictiveResponseEngine(adapter, clf, rel)
    return StreamingPredictiveBridge(StreamingCommandParser(None, fallback_parser, enabled=False),
                                     engine, StatusManager(tts), clf,
                                     AsyncExecutionPipeline(adapter))


def build_gpu_processor(cfg: Config, nats, device: str = "cuda:0", tts=None, *, skills=None,
                        llm=None, bridge: bool = True):
    """On-device STT -> constrained intent decode -> queue (one GPU), the
    bridge on that decode, and the reply voice (``tts``: "auto" builds it from
    ``HUB_TTS_BACKEND``). ``llm``: a prebuilt engine (the tensor-parallel
    leader, ``parallel/tp_serving.py``). Speech is progressive (phrases from
    the live decode) when ``STREAMING_ENABLED``."""
    from .engine.llm_engine import LLMEngine
    from .engine.pipeline import VoicePipeline
    from .engine.stt_engine import STTEngine
    from .streaming.components import tts_options_from
    from .transport.voice_processor import GPUVoiceProcessor
    g = cfg.gpu
    scfg, lcfg = g.stt_config(), g.llm_config()
    sw = lw = None
    if g.stt_checkpoint or (g.llm_checkpoint and llm is None):
        from .models import loader
        sw = loader.load_whisper(scfg, g.stt_checkpoint, device) if g.stt_checkpoint else None
        lw = loader.load_llama(lcfg, g.llm_checkpoint, device) if (g.llm_checkpoint and llm is None) \
            else None
    stt = STTEngine(scfg, device, seed=g.seed, max_batch=g.max_batch, use_graphs=g.use_graphs,
                    weights=sw, tokenizer=g.tokenizer("stt", scfg.vocab_size),
                    language=cfg.stt.language)
    if llm is None:
        llm = LLMEngine(lcfg, device, seed=g.seed, max_seqs=g.max_batch, weights=lw,
                        max_seq_len=g.max_seq_len, block_size=g.kv_block, use_graphs=g.use_graphs,
                        tokenizer=g.tokenizer("llm", lcfg.vocab_size))
    if tts == "auto":
        tts = build_tts(cfg, device)
    pipe = VoicePipeline(stt, llm, nats)
    pipe.warmup()
    if tts is not None and hasattr(tts, "warmup_graphs"):
        tts.warmup_graphs()         # VITS graph buckets of typical replies
    sc = cfg.streaming
    proc = GPUVoiceProcessor(pipe, tts=tts, max_batch=min(g.max_batch, 64),
                             bridge=build_bridge(skills, tts) if bridge else None,
                             bridge_timeout=cfg.arbitration.bridge_timeout,
                             progressive=sc.enabled, tts_options=tts_options_from(cfg),
                             tts_format=cfg.tts.response_format,
                             max_buffer_time=sc.max_buffer_time,
                             max_tokens_per_phrase=sc.max_tokens_per_phrase)
    if llm.tp.world > 1 and g.tp_fallback_model != "none":
        # a failed TP group degrades to a single-GPU engine
        from .parallel.tp_serving import TPFailover
        proc.tp_failover = TPFailover(proc, g.tp_fallback_config(), device, seed=g.seed,
                                      max_seqs=g.max_batch, max_seq_len=g.max_seq_len,
                                      block_size=g.kv_block,
                                      checkpoint=g.tp_fallback_checkpoint,
                                      require_checkpoint=bool(g.llm_checkpoint)).attach(llm)
    return proc


async def build_dp_processor(cfg: Config, n_gpus: int, nats_url: str = "", *,
                             device: str = "cuda", skills_dir: str = "./skills",
                             skills_config_store: str = "./data/skills", **spec_kw):
    """One worker process per GPU behind the least-loaded router (D1). Each
    worker builds the full per-GPU composition (``build_gpu_processor``: STT,
    constrained decode, command queue over its own connection to the hub's
    NATS broker at ``nats_url``, bridge, reply voice, progressive speech).
    ``device``: "cuda" (worker r on cuda:r), "cuda:0" (every worker on one
    GPU: the shared-GPU rehearsal) or "cpu"."""
    from .parallel.dp_serving import DPVoiceProcessor
    spec = {"device": device, "cfg": cfg, "nats_url": nats_url, "seed": cfg.gpu.seed,
            "skills_dir": skills_dir, "skills_config_store": skills_config_store, **spec_kw}
    dp = DPVoiceProcessor(spec, n_gpus)
    await dp.start()
    return dp


async def build_service_processor(cfg: Config, nats, tts=None):
    """Reference path: external STT + Ollama parser (+ TTS)."""
    from .llm.command_parser import CommandParser, OllamaBackend
    from .llm.stt_client import STTClient
    from .transport.voice_processor import ServiceVoiceProcessor
    stt = STTClient(cfg.stt.url, cfg.stt.language)
    parser = CommandParser(OllamaBackend(cfg.ollama.url, cfg.ollama.model))
    return ServiceVoiceProcessor(stt, parser, nats=nats, tts=tts)


class HubServer:
    def __init__(self, cfg: Config, *, processor=None, nats: NATSService | None = None,
                 streaming=None, skills_dir: str = "./skills",
                 skills_config_store: str = "./data/skills", transcript_hints=None):
        self.cfg = cfg
        self.database = Database(cfg.server.db_path)
        self.events = VoiceEventsStore(self.database)
        self.nats = nats
        self.processor = processor
        self.streaming = streaming
        self.skills = SkillManager(SkillManagerConfig(skills_dir=skills_dir,
                                                      config_store=skills_config_store),
                                   DefaultSkillLoader(skills_root=skills_dir))
        self.audio_service: AudioService | None = None
        self.grpc_server = None
        self.http_runner: web.AppRunner | None = None
        self.http_port = 0
        self.grpc_port = 0
        self._embedded_broker = None
        self.transcript_hints = transcript_hints     # synthetic load only (AudioService)

    # ------------------------------------------------------------------ wiring
    def app(self) -> web.Application:
        app = web.Application()
        app.router.add_get("/health", self.handle_health)
        app.add_routes(VoiceEventsHandler(self.events).routes())
        app.add_routes(SkillsHandler(self.skills).routes())
        app.add_routes(StreamingHandler(self.streaming).routes())
        app.add_routes(MetricsHandler(self).routes())
        return app

    async def handle_health(self, req: web.Request) -> web.Response:
        log.info("Health check received")
        return web.Response(text="ok\n", content_type="text/plain")

    async def _connect_nats(self) -> None:
        url = self.cfg.nats.url
        if self.nats is None:
            if url == "embedded":
                from .messaging.nats_server import NATSServer
                self._embedded_broker = await NATSServer().start()
                url = self._embedded_broker.url
            self.nats = NATSService(url, self.cfg.nats.reconnect_wait)
        if not self.nats.is_connected():
            try:
                await self.nats.connect()
            except Exception as e:  # noqa: BLE001 - hub keeps serving without the bus
                log.warning("Cannot connect to NATS: %s (events will not be published)", e)

    async def _check_tts(self) -> None:
        """The reference tests the TTS service at start-up and, with
        ``TTS_FALLBACK_ENABLED``, keeps serving text-only if it is down
        (``audio_service.go:182-195``)."""
        tts = getattr(self.processor, "tts", None)
        test = getattr(tts, "test_connection", None)
        if test is None:
            return
        try:
            await test()
        except Exception as e:  # noqa: BLE001
            if not self.cfg.tts.fallback_enabled:
                raise RuntimeError(f"failed to connect to TTS service: {e}") from e
            log.warning("TTS service unavailable, continuing without speech: %s", e)
            self.processor.tts = None
            if hasattr(self.processor, "progressive"):
                self.processor.progressive = False

    async def start(self, host: str | None = None, http_port: int | None = None,
                    grpc_port: int | None = None) -> None:
        import grpc

        from .transport.audio_proto import add_audio_service
        await self._connect_nats()
        await self.skills.register_plugin(LightsSkill())
        await self.skills.start()
        publisher = AudioStreamPublisher(self.nats.conn) if self.nats and self.nats.conn else None
        if hasattr(self.processor, "attach_publisher"):
            self.processor.attach_publisher(publisher)   # progressive per-phrase speech
        await self._check_tts()
        if (self.streaming is None and self.cfg.streaming.enabled
                and hasattr(self.processor, "attach_streaming")):
            # streaming_constructor.go:38-126, composed into the served hub: the
            # processor's progressive replies are the streaming sessions
            from .streaming.components import StreamingComponents
            self.streaming = StreamingComponents.for_processor(self.cfg, self.processor)
        if self.streaming is not None and hasattr(self.processor, "attach_streaming"):
            self.processor.attach_streaming(self.streaming)
        a = self.cfg.arbitration
        self.audio_service = AudioService(
            self.processor, window_duration=a.window, scope=a.scope, relay_groups=a.relay_groups,
            single_relay_bypass=a.single_relay_bypass,
            end_of_speech_wait=a.end_of_speech_wait, events_store=self.events,
            audio_publisher=publisher, confirmation_enabled=a.confirmation_enabled,
            transcript_hints=self.transcript_hints)
        host = host if host is not None else self.cfg.server.host
        self.grpc_server = grpc.aio.server()
        add_audio_service(self.grpc_server, self.audio_service)
        gport = self.cfg.server.grpc_port if grpc_port is None else grpc_port
        self.grpc_port = self.grpc_server.add_insecure_port(f"{host}:{gport}")
        await self.grpc_server.start()
        log.info("gRPC server listening on :%d", self.grpc_port)
        self.http_runner = web.AppRunner(self.app())
        await self.http_runner.setup()
        site = web.TCPSite(self.http_runner, host,
                           self.cfg.server.port if http_port is None else http_port)
        await site.start()
        self.http_port = site._server.sockets[0].getsockname()[1]  # type: ignore[union-attr]
        log.info("HTTP server listening on :%d", self.http_port)
        # the start-up objects (models, protobuf classes, the composition) are
        # long-lived: move them out of the cyclic GC's generations and collect
        # young objects less often, so full collections do not stall the event
        # loop in the middle of relay traffic (front-end p99, docs/PERF.md)
        import gc
        gc.collect()
        gc.freeze()
        gc.set_threshold(50000, 20, 100)

    async def stop(self) -> None:
        stop = getattr(self.processor, "close", None)
        if stop is not None:
            await stop()
        if self.grpc_server is not None:
            await self.grpc_server.stop(1.0)
        if self.http_runner is not None:
            await self.http_runner.cleanup()
        await self.skills.stop()
        if self.streaming is not None:
            await self.streaming.shutdown()
        if self.nats is not None:
            await self.nats.close()
        if self._embedded_broker is not None:
            await self._embedded_broker.stop()
        self.database.close()

    async def serve_forever(self) -> None:
        await self.start()
        try:
            while True:
                await asyncio.sleep(3600)
        finally:
            await self.stop()
