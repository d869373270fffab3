"""Tensor-parallel serving of the intent decoder (BASELINE config 5: Llama-3-70B
at TP=8 on one 8-GPU node).

One process per GPU (``torchrun --nproc-per-node N``). Rank 0 is the hub: it
owns the gRPC / HTTP / NATS front end, the Whisper STT and VITS TTS engines and
the LEADER of the tensor-parallel LLM engine; ranks 1..N-1 run FOLLOWER engines
that replay the leader's scheduler iterations (``parallel/tp_control.py``).
Every decode step is the fused TP step (``models/llama.py``): column-parallel
qkv / gate|up, row-parallel o / down whose f32 partials one custom IPC kernel
reduce-scatters onto the replicated residual stream, and a vocab-parallel
argmax combine - 2 x n_layers + 1 one-hop collectives over the xGMI mesh per
step, captured in the step's HIP graph.

The process group is gloo (CPU): it only carries start-up traffic (IPC handles,
barriers); every data-plane collective is the custom kernel, so no RCCL
communicator (and none of its streams) exists in a TP job.

Launch (one 8-GPU node, config 5)::

    HUB_TP=8 HUB_LLM_MODEL=llama3-70b HUB_STT_MODEL=whisper-large-v3 \\
      torchrun --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \\
      --master-port 29533 -m loqa_hub_amd.cli.main
    # benchmark of the same layout:
    torchrun --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \\
      --master-port 29533 scripts/bench_configs.py --config 5 --tp 8
"""
from __future__ import annotations

import logging
import os
import threading
import time

import torch
import torch.distributed as dist

from .dist import DistInfo

log = logging.getLogger("loqa.tp")


def init_tp(tp: int) -> DistInfo:
    """The TP process group from the torchrun environment (gloo); the GPU is
    ``cuda:LOCAL_RANK``. Fails loudly when the job was not launched with
    ``--nproc-per-node tp``."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != tp:
        raise RuntimeError(f"HUB_TP={tp} needs {tp} ranks: launch with torchrun "
                           f"--nproc-per-node {tp} (WORLD_SIZE is {world})")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    torch.cuda.set_device(local)
    if not dist.is_initialized():
        dist.init_process_group("gloo", rank=rank, world_size=world)
    return DistInfo(rank, local, world, torch.device("cuda", local), "gloo")


def build_tp_llm(lcfg, info: DistInfo, *, seed: int = 0, max_seqs: int = 64,
                 max_seq_len: int = 1024, block_size: int = 16, use_graphs: bool = True,
                 compact: bool = False, checkpoint: str = "", tokenizer=None):
    """This rank's engine of the TP group: custom all-reduce, Megatron shard of
    the seeded (or ``checkpoint``) weights, and the lock-step control ring."""
    from ..engine.llm_engine import LLMEngine
    from ..models.llama import TPGroup
    from .tp_control import TPControl, control_tag
    tp = TPGroup.create(info.rank, info.world, dist.group.WORLD, device=info.device)
    weights = None
    if checkpoint:
        from ..models import loader
        weights = loader.load_llama(lcfg, checkpoint, info.device, tp=tp)
    eng = LLMEngine(lcfg, info.device, seed=seed, max_seqs=max_seqs, max_seq_len=max_seq_len,
                    block_size=block_size, tp=tp, use_graphs=use_graphs, weights=weights,
                    compact=compact, tokenizer=tokenizer)
    eng.tp_ctl = TPControl(info.rank, info.world, control_tag(), dist.group.WORLD)
    eng.tp_ctl.start_heartbeat()
    return eng


def run_follower(eng) -> dict:
    """A follower rank: capture the decode graphs (in step with the leader),
    then replay the leader's iterations until it stops."""
    eng.warmup_graphs()
    log.info("TP follower rank %d serving", eng.tp.rank)
    eng.follow()
    torch.cuda.synchronize()
    stats = dict(eng.stats)
    if eng.tp.car is not None and eng.tp.car.error():
        raise RuntimeError(f"TP rank {eng.tp.rank}: a collective timed out")
    eng.tp_ctl.close()
    return stats


class TPFailover:
    """Degradation of a failed tensor-parallel group ("TP=8 ...
    fall back to the 8B DP path and flag it in metrics"; the reference's own
    discipline is to fall back to a working path and tell the user -
    ``audio_service.go:641-664`` bridge -> parser, ``:261-287`` service retry).

    The leader engine calls ``on_failure`` from its scheduler thread when a
    collective times out, a follower stops heart-beating, or an iteration
    fails (``LLMEngine._tp_fail``): its in-flight and queued requests have
    already failed (the hub answers them with the STT-failed reply), the
    followers got the stop record. This builds the fallback engine
    (``HUB_TP_FALLBACK_MODEL``, default Llama-3-8B, on the leader's GPU: it
    fits beside the 70B shard in 288 GB) on a thread of its own and swaps it
    into the voice pipeline; until then every utterance fails fast. The
    fallback decodes eagerly (no graph capture while the STT engine serves).
    ``stats``: ``tp_degraded`` (1 once failed), ``tp_fallback_ready``.

    Weights: ``checkpoint`` (``HUB_TP_FALLBACK_CHECKPOINT``, with the tokenizer
    in / beside it or ``tokenizer``) loads a real model. Without one the
    fallback is the seeded random-init model, which is only acceptable when the
    TP group itself serves random-init weights: ``require_checkpoint`` (set by
    the hub when ``HUB_LLM_CHECKPOINT`` is) makes the failover fail CLOSED -
    utterances keep failing with the STT-failed reply and
    ``tp_fallback_refused`` is set - instead of publishing a random model's
    commands on ``loqa.devices.commands.*``."""

    def __init__(self, processor, lcfg, device, *, seed: int = 0, max_seqs: int = 64,
                 max_seq_len: int = 1024, block_size: int = 16, build=None,
                 checkpoint: str = "", tokenizer=None, require_checkpoint: bool = False):
        self.processor, self.lcfg, self.device = processor, lcfg, device
        self.kw = dict(seed=seed, max_seqs=max_seqs, max_seq_len=max_seq_len,
                       block_size=block_size, use_graphs=False)
        self._build = build
        self.checkpoint, self.tokenizer = checkpoint, tokenizer
        self.require_checkpoint = require_checkpoint
        self.error = ""
        self.t_failed = 0.0
        self.ready = threading.Event()
        self._lock = threading.Lock()

    def attach(self, leader) -> "TPFailover":
        leader.on_tp_failure = self.on_failure
        return self

    def on_failure(self, err: Exception) -> None:
        with self._lock:
            if self.t_failed:
                return
            self.t_failed = time.monotonic()
            self.error = str(err)
        st = self.processor.stats
        st["tp_degraded"] = 1
        st["tp_fallback_ready"] = 0
        if self._build is None and self.require_checkpoint and not self.checkpoint:
            st["tp_fallback_refused"] = 1
            log.error("tensor-parallel group failed (%s) and no fallback checkpoint is set "
                      "(HUB_TP_FALLBACK_CHECKPOINT): the primary serves a checkpoint, so the hub "
                      "will not fall back to random-init weights - utterances fail until restart",
                      err)
            return
        log.error("tensor-parallel group failed (%s): serving falls back to %s on %s",
                  err, self.lcfg.name, self.device)
        threading.Thread(target=self._swap, name="tp-failover", daemon=True).start()

    def _swap(self) -> None:
        try:
            if self._build is not None:
                eng = self._build()
            else:
                from ..engine.llm_engine import LLMEngine
                weights, tok = None, self.tokenizer
                if self.checkpoint:
                    from ..engine.tokenizer import find_tokenizer, load_tokenizer
                    from ..models import loader
                    weights = loader.load_llama(self.lcfg, self.checkpoint, self.device)
                    if tok is None and find_tokenizer(self.checkpoint):
                        tok = load_tokenizer(self.checkpoint, self.lcfg.vocab_size)
                eng = LLMEngine(self.lcfg, self.device, weights=weights, tokenizer=tok, **self.kw)
            old = self.processor.pipeline.llm
            self.processor.pipeline.llm = eng
            self.processor.stats["tp_fallback_ready"] = 1
            self.processor.stats["tp_failover_s"] = round(time.monotonic() - self.t_failed, 3)
            self.ready.set()
            log.warning("fallback LLM engine %s serving (%.1f s after the TP failure)",
                        self.lcfg.name, time.monotonic() - self.t_failed)
            try:
                if old.tp_ctl is not None:
                    old.tp_ctl.close()
            except Exception:  # noqa: BLE001
                pass
        except Exception:  # noqa: BLE001
            log.exception("building the fallback LLM engine failed: the hub cannot parse commands")
