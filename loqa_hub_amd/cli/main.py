"""Hub entry point (``cmd/main.go:29-54``): logging, configuration, server.

    python -m loqa_hub_amd.cli.main            # env-configured

Backends follow ``HUB_*``: with a visible GPU and ``HUB_LLM_BACKEND=gpu``
(default) the on-device pipeline serves STT + intent parsing on ``cuda:0``;
otherwise the reference's external services (STT_URL, OLLAMA_URL, TTS_URL).
With ``HUB_NUM_GPUS`` (or ``HUB_DP``) > 1 the hub front-end stays in this
process and spawns one worker process per GPU behind the least-loaded router
with crash / hang re-routing (``parallel/dp_serving.py``).
"""
from __future__ import annotations

import asyncio
import logging
import sys

from .. import config as cfgmod
from ..utils import logging as hublog

log = logging.getLogger("loqa.main")


async def run(cfg) -> None:
    from ..server import (HubServer, build_dp_processor, build_gpu_processor,
                          build_service_processor)
    server = HubServer(cfg)
    await server._connect_nats()
    processor = None
    use_gpu = cfg.gpu.llm_backend == "gpu" and cfg.gpu.stt_backend == "gpu"
    if use_gpu:
        import torch
        n = torch.cuda.device_count()
        want = cfg.gpu.dp or cfg.gpu.num_gpus or 1
        if n > 1 and want > 1:
            processor = await build_dp_processor(cfg, min(n, want))
        elif n > 0:
            processor = build_gpu_processor(cfg, server.nats)
        else:
            log.warning("no GPU visible; using the external STT/LLM services")
    if processor is None:
        processor = await build_service_processor(cfg, server.nats)
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
    try:
        asyncio.run(run(cfg))
    except KeyboardInterrupt:
        pass
    return 0


if __name__ == "__main__":
    sys.exit(main())
