"""``/api/metrics``: Prometheus text exposition of the hub's counters (audio
service arbitration, GPU engines, skills, NATS). The reference exposes no
metrics endpoint; this is additive."""
from __future__ import annotations

from aiohttp import web


def _line(name: str, value, labels: dict | None = None, help_: str = "") -> str:
    lab = ""
    if labels:
        lab = "{" + ",".join(f'{k}="{v}"' for k, v in sorted(labels.items())) + "}"
    return f"{name}{lab} {float(value)}"


class MetricsHandler:
    def __init__(self, server):
        self.server = server

    def routes(self) -> list[web.RouteDef]:
        return [web.get("/api/metrics", self.metrics), web.get("/api/trace", self.trace)]

    def collect(self) -> list[str]:
        s = self.server
        out = []
        if s.audio_service is not None:
            for k, v in s.audio_service.stats.items():
                out.append(_line("loqa_audio_" + k + "_total", v))
            out.append(_line("loqa_audio_active_streams", len(s.audio_service.active_streams)))
        if s.skills is not None:
            out.append(_line("loqa_skills_loaded", len(s.skills.skills)))
        proc = getattr(s, "processor", None)
        for k, v in (getattr(proc, "stats", None) or {}).items():
            out.append(_line("loqa_processor_" + k + "_total", v))
        dpm = proc.metrics() if hasattr(proc, "metrics") else None
        if dpm is not None:  # data-parallel workers (one per GPU)
            out.append(_line("loqa_gpu_workers_healthy", dpm["healthy"]))
            out.append(_line("loqa_gpu_worker_failures_total", len(dpm["failures"])))
            for w in dpm["workers"]:
                lab = {"rank": w["rank"]}
                out.append(_line("loqa_gpu_worker_healthy", int(w["healthy"]), lab))
                out.append(_line("loqa_gpu_worker_queue_depth", w["queued"], lab))
                out.append(_line("loqa_gpu_worker_utterances_total", w["done"], lab))
                for k, v in w["stats"].items():
                    if isinstance(v, (int, float)):
                        out.append(_line("loqa_gpu_worker_" + k + "_total", v, lab))
        pipe = getattr(proc, "pipeline", None)
        if pipe is not None:
            for k, v in pipe.llm.stats.items():
                out.append(_line("loqa_llm_" + k, v))
            for k, v in pipe.stt.stats.items():
                out.append(_line("loqa_stt_" + k, v))
        from ..utils.tracing import tracer
        for stage, st in tracer().summary().items():
            lab = {"stage": stage}
            out.append(_line("loqa_stage_count", st["count"], lab))
            out.append(_line("loqa_stage_p50_ms", st["p50_ms"], lab))
            out.append(_line("loqa_stage_p99_ms", st["p99_ms"], lab))
        nats = s.nats.stats() if s.nats is not None and s.nats.conn is not None else None
        if nats is not None:
            for k, v in vars(nats).items():
                out.append(_line("loqa_nats_" + k, v))
        return out

    async def trace(self, req: web.Request) -> web.Response:
        """Chrome-trace JSON of the recent per-stage spans (load in Perfetto)."""
        from ..utils.tracing import tracer
        return web.Response(text=tracer().chrome_trace(), content_type="application/json")

    async def metrics(self, req: web.Request) -> web.Response:
        return web.Response(text="\n".join(self.collect()) + "\n",
                            content_type="text/plain", charset="utf-8")
