"""Hub entry point (``cmd/main.go:29-54``): logging, configuration, server.

    python -m loqa_hub_amd.cli.main            # env-configured

Backends follow ``HUB_*``: with a visible GPU and ``HUB_LLM_BACKEND=gpu``
(default) the on-device pipeline serves STT + intent parsing on ``cuda:0``;
otherwise the reference's external services (STT_URL, OLLAMA_URL, TTS_URL).
With ``HUB_NUM_GPUS`` (or ``HUB_DP``) > 1 the hub front-end stays in this
process and spawns one worker process per GPU behind the least-loaded router
with crash / hang re-routing (``parallel/dp_serving.py``). With ``HUB_TP`` > 1
the job is launched by torchrun with one process per GPU: rank 0 serves the
hub with the tensor-parallel LLM leader, the other ranks are followers
(``parallel/tp_serving.py``). The reply voice follows ``HUB_TTS_BACKEND``
(gpu: on-device VITS; http: the OpenAI-compatible ``TTS_URL``; none).
"""
from __future__ import annotations

import asyncio
import logging
import sys

from .. import config as cfgmod
from ..utils import logging as hublog

log = logging.getLogger("loqa.main")


def _tp_engine(cfg):
    """HUB_TP > 1: this rank's TP engine (rank 0: the leader, served below)."""
    from ..parallel.tp_serving import build_tp_llm, init_tp
    g = cfg.gpu
    info = init_tp(g.tp)
    lcfg = g.llm_config()
    eng = build_tp_llm(lcfg, info, seed=g.seed, max_seqs=g.max_batch,
                       max_seq_len=g.max_seq_len, block_size=g.kv_block,
                       use_graphs=g.use_graphs, checkpoint=g.llm_checkpoint,
                       tokenizer=g.tokenizer("llm", lcfg.vocab_size))
    return info, eng


async def run(cfg, tp_leader=None) -> None:
    from ..server import (HubServer, build_dp_processor, build_gpu_processor, build_service_processor,
                          build_tts)
    server = HubServer(cfg)
    await server._connect_nats()
    processor = None
    use_gpu = cfg.gpu.llm_backend == "gpu" and cfg.gpu.stt_backend == "gpu"
    if tp_leader is not None:
        info, eng = tp_leader
        processor = build_gpu_processor(cfg, server.nats, device=str(info.device), tts="auto",
                                        skills=server.skills, llm=eng)
    elif use_gpu:
        import torch
        n = torch.cuda.device_count()
        want = cfg.gpu.dp or cfg.gpu.num_gpus or 1
        if n > 1 and want > 1:
            processor = await build_dp_processor(
                cfg, min(n, want), server.nats.url if server.nats is not None else "")
        elif n > 0:
            processor = build_gpu_processor(cfg, server.nats, tts="auto", skills=server.skills)
        else:
            log.warning("no GPU visible; using the external STT/LLM services")
    if processor is None:
        tts = build_tts(cfg) if cfg.gpu.tts_backend in ("http", "openai") else None
        processor = await build_service_processor(cfg, server.nats, tts=tts)
    server.processor = processor
    log.info("starting loqa hub (http :%d, grpc :%d)", cfg.server.port, cfg.server.grpc_port)
    await server.serve_forever()


def main(argv=None) -> int:
    hublog.initialize()
    try:
        cfg = cfgmod.load()
    except cfgmod.ConfigError as e:
        log.error("Failed to load configuration: %s", e)
        return 1
    hublog.initialize(cfg.logging.level, cfg.logging.format)
    tp_leader = None
    if cfg.gpu.tp > 1:
        info, eng = _tp_engine(cfg)
        if info.rank != 0:
            from ..parallel.tp_serving import run_follower
            run_follower(eng)
            return 0
        tp_leader = (info, eng)
    try:
        asyncio.run(run(cfg, tp_leader))
    except KeyboardInterrupt:
        pass
    return 0


if __name__ == "__main__":
    sys.exit(main())
