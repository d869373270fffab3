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
                 compact: bool = False, checkpoint: str = ""):
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
                    compact=compact)
    eng.tp_ctl = TPControl(info.rank, info.world, control_tag(), dist.group.WORLD)
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
