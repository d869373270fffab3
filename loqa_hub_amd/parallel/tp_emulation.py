"""Tensor-parallel emulation in ONE process (bitwise TP checks).

``TPEmulation(cfg, device, world)`` holds the ``world`` Megatron shards of the
model (the same counter-based init as a real TP rank builds) with one KV cache
per shard, and runs the fused TP decode step (``LlamaModel.forward_decode_fused``
at tp > 1) shard by shard, layer by layer: each shard's qkv / attention / o
partial, then the residual all-reduce of the W partials through
``tp_emul_resid_kernel`` - phase 1 of the IPC kernel's arithmetic, shared code
(``car_resid_math``) - then each shard's gate|up / down partial, and so on; the
logits stay per shard and the vocab-parallel argmax combine is the exact
(max logit, lowest id) rule. A real TP=W run (W processes, IPC collectives,
lock-step graphs) must therefore produce BITWISE the same logit shards and
tokens - any difference is a sharding, data-movement or synchronisation bug,
not rounding. (Decode-GEMM tuning must be off on both sides, LOQA_NO_TUNE=1,
so every shard runs the default split configuration.)
"""
from __future__ import annotations

import torch

from .. import ops
from ..engine.llm_engine import LLMEngine
from ..models.llama import TPGroup
from .custom_allreduce import resid_blocks_for


class _EmulGroup(TPGroup):
    """A shard's TP context inside the emulation: no collectives of its own."""

    def __init__(self, rank: int, world: int):
        super().__init__(rank, world, None, None)


class TPEmulation:
    def __init__(self, cfg, device, world: int, *, seed: int = 0, max_seqs: int = 8,
                 max_seq_len: int = 512):
        self.world = world
        self.cfg = cfg
        self.engines = [LLMEngine(cfg, device, seed=seed, max_seqs=max_seqs, max_seq_len=max_seq_len,
                                  tp=_EmulGroup(r, world), use_graphs=False)
                        for r in range(world)]
        self.scratch = self.engines[0].scratch
        self.nblk = resid_blocks_for(cfg.d_model, world)
        self.device = self.engines[0].device

    # every shard's KV pool sees the same sequence operations, so the step
    # metadata of shard 0 addresses every shard's cache identically
    def add_seq(self, seq_id: int) -> None:
        for e in self.engines:
            e.kv.pool.add_seq(seq_id, [])

    def free_seq(self, seq_id: int) -> None:
        for e in self.engines:
            e.kv.pool.free_seq(seq_id)

    def meta(self, reqs, feeds, B_pad: int, T_pad: int):
        metas = [e._meta(reqs, feeds, True, B_pad, T_pad) for e in self.engines]
        max_q, max_ctx, host = metas[0]
        for _, _, h in metas[1:]:
            for k in host:
                assert (h[k] == host[k]).all(), f"shard metadata diverged: {k}"
        dev = self.engines[0]._to_device(host)
        return self.engines[0]._build_meta(dev, max_q, max_ctx, True), dev

    def resid(self, residual: torch.Tensor, partials: torch.Tensor) -> None:
        Mpad, d = residual.shape
        ops._lib.check(ops._lib.kernels().loqa_tp_emul_resid(
            partials.data_ptr(), residual.data_ptr(), self.scratch.rowsq.data_ptr(), Mpad, d,
            self.world, self.nblk, ops._lib.stream_ptr(residual)), "tp_emul_resid")
        self.scratch.stat_tiles = self.world * self.nblk

    def forward_decode_fused(self, meta) -> list[torch.Tensor]:
        """The TP decode step of ``LlamaModel.forward_decode_fused`` for all
        shards; returns each shard's f32 logits [rows, V / world]."""
        cfg, W = self.cfg, self.world
        ws = [e.weights for e in self.engines]
        w0, scratch = ws[0], self.scratch
        H, Hkv, D, d = w0.h, w0.hkv, cfg.head_dim, cfg.d_model
        Mpad = meta.tokens.numel()
        if ops.FUSED_EMBED and w0.embed.shape[0] == cfg.vocab_size and meta.tokens.dtype == torch.int32:
            residual = ops.embed_stats(meta.tokens, w0.embed, scratch)
        else:
            residual = self.engines[0].model.embed(meta.tokens).contiguous()
            scratch.seed_stats(residual, sums=False)
        num_splits, split_keys = ops.decode_attn_splits(meta.max_ctx, meta.ctx_lens.numel() * Hkv,
                                                        self.engines[0].attn_split_keys,
                                                        getattr(w0, "max_wgs", None))
        grouped = (H // Hkv) * meta.max_q <= 128
        partials = torch.empty(W, Mpad, d, dtype=torch.float32, device=residual.device)
        for li in range(cfg.n_layers):
            for r, e in enumerate(self.engines):
                P = ws[r].decode_layers[li]
                q = torch.empty(Mpad, H * D, dtype=torch.bfloat16, device=residual.device)
                ops.skinny_fused(residual, P["wqkv_f"], "rope", scratch, norm=True, eps=cfg.norm_eps,
                                 positions=meta.positions, cos_sin=ws[r].cos_sin, q_out=q,
                                 k_cache=e.kv.k[li], v_cache=e.kv.v[li], slots=meta.slots,
                                 n_heads=H, n_kv=Hkv, head_dim=D)
                attn = ops.attention(q, e.kv.k[li], e.kv.v[li], meta.cu_q, n_heads=H, n_kv=Hkv,
                                     head_dim=D, causal=True, max_q=meta.max_q,
                                     ctx_lens=meta.ctx_lens, block_tables=meta.block_tables,
                                     grouped=grouped, split_keys=split_keys,
                                     num_splits=num_splits if grouped else 1,
                                     workspace=e.attn_ws, max_k=meta.max_ctx)
                ops.skinny_fused(attn, P["wo"], "act", scratch, out=partials[r], act="f32")
            self.resid(residual, partials)
            for r, e in enumerate(self.engines):
                P = ws[r].decode_layers[li]
                a = ops.skinny_fused(residual, P["w_gate_up_f"], "silu", scratch, norm=True,
                                     eps=cfg.norm_eps)
                ops.skinny_fused(a, P["w_down"], "act", scratch, out=partials[r], act="f32")
            self.resid(residual, partials)
        if ops.FUSED_EMBED:
            hf = ops.rmsnorm(residual, w0.final_norm, cfg.norm_eps, row_idx=meta.logit_idx)
        else:
            hf = ops.rmsnorm(residual.index_select(0, meta.logit_idx), w0.final_norm, cfg.norm_eps)
        return [ops.skinny_gemm(hf, w.lm_head_p, 1,
                                max_wgs=getattr(w, "max_wgs", ops.MAX_DECODE_WGS))[0][:, :w.v]
                for w in ws]

    @staticmethod
    def argmax_combine(shard_logits: list[torch.Tensor], shard_idx: list[torch.Tensor]) -> torch.Tensor:
        """The vocab-parallel combine rule of ``car_argmax_kernel``: the
        largest logit over the shards' picks, ties to the lowest token id."""
        B = shard_idx[0].numel()
        out = torch.full((B,), -1, dtype=torch.int32)
        for b in range(B):
            best = None
            for r, (lg, ix) in enumerate(zip(shard_logits, shard_idx)):
                i = int(ix[b])
                if i < 0:
                    continue
                v = float(lg[b, i])
                tok = i + r * lg.shape[1]
                if best is None or v > best[0] or (v == best[0] and tok < best[1]):
                    best = (v, tok)
            if best is not None:
                out[b] = best[1]
        return out
