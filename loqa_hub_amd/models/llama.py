"""Llama-family decoder (TinyLlama, Llama-3.2-1B/3B, Llama-3-8B/70B) for the
intent parser that replaces the reference's Ollama call
(``command_parser.go:223-266``, ``streaming_command_parser.go:339-371``).

Layout is MI355X-first rather than HF-module-first:

* fused QKV weight [(H + 2 Hkv) D, d] and fused gate|up weight [2F, d] so each
  layer is 4 GEMMs (hipBLASLt) + 4 fused HIP kernels (rmsnorm+residual,
  rope+paged-KV-append, flash/paged attention, SwiGLU);
* the residual stream is updated inside the norm kernel;
* activations are a flat [T, d] token batch (continuous batching), sequence
  structure lives only in the attention metadata;
* tensor parallel: QKV/gate-up column-sharded by head / ffn slice, O/down
  row-sharded with one all-reduce each, vocab-parallel lm_head with a
  (max, argmax) combine.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch

from .. import ops
from ..ops.reference import rope_cos_sin
from .configs import LlamaConfig


@dataclass
class StepMeta:
    """Device-side metadata of one forward over a flat token batch."""
    tokens: torch.Tensor        # [T] int32
    positions: torch.Tensor     # [T] int32
    slots: torch.Tensor         # [T] int32 (KV slot, -1 = padding row)
    cu_q: torch.Tensor          # [B+1] int32
    ctx_lens: torch.Tensor      # [B] int32 (tokens in cache after this step)
    block_tables: torch.Tensor  # [B, max_blocks] int32
    logit_idx: torch.Tensor     # [B] int64 rows whose logits are needed
    max_q: int
    max_ctx: int
    decode: bool                # grouped (small-q) attention path
    # a mixed prompt pass whose leading sequences are live decoders: (their
    # count, their rows, their longest feed, their longest context, the prompt
    # sequences' cu_q relative to the first prompt row) - the two groups get
    # their own attention launches (grouped decode attention reads each kv
    # head's cache once; the flash prefill kernel would re-read it per q head)
    split: tuple | None = None


class TPGroup:
    """Tensor-parallel context; world 1 = no-op.

    On GPUs every collective of a TP decode step is a custom IPC kernel
    (``parallel/custom_allreduce.py``): the row-parallel o / down all-reduce fused
    with the residual add and the next norm's row statistics, and the
    vocab-parallel argmax combine. On the CPU (gloo) the same step runs through
    ``dist`` collectives, which is what the CPU test tier exercises."""

    def __init__(self, rank: int = 0, world: int = 1, group=None, allreduce=None):
        self.rank, self.world, self.group = rank, world, group
        self._allreduce = allreduce

    @classmethod
    def create(cls, rank: int, world: int, group=None, device=None,
               custom_allreduce: bool = True) -> "TPGroup":
        """TP group; on GPUs the decode/prefill all-reduces use the one-shot IPC
        kernel (parallel/custom_allreduce.py) with RCCL as the fallback."""
        ar = None
        if world > 1 and custom_allreduce and device is not None and \
                torch.device(device).type == "cuda":
            from ..parallel.custom_allreduce import CustomAllReduce
            ar = CustomAllReduce(group)
            # every collective checked against the host reduction before the
            # group serves (raises on every rank on a mismatch)
            ar.self_test()
        return cls(rank, world, group, ar)

    @property
    def car(self):
        """The custom all-reduce (None: dist collectives)."""
        return self._allreduce

    def all_reduce_(self, x: torch.Tensor) -> torch.Tensor:
        if self.world == 1:
            return x
        if self._allreduce is not None:
            return self._allreduce(x)
        import torch.distributed as dist
        dist.all_reduce(x, group=self.group)
        return x

    def partial_out(self, which: int, rows: int, cols: int, device):
        """Where a row-parallel GEMM writes its f32 partial (the IPC input
        buffer on GPUs, a plain tensor for the dist path)."""
        if self._allreduce is not None:
            return self._allreduce.inbuf(which, rows, cols)
        return torch.empty(rows, cols, dtype=torch.float32, device=device)

    def resid_epilogue(self, which: int, partial, residual: torch.Tensor, scratch) -> None:
        """residual += sum over ranks of ``partial``; the row sums of squares
        of the new residual go to ``scratch`` for the next norm prologue."""
        if self._allreduce is not None:
            nb = self._allreduce.resid_blocks(residual.shape[1])
            self._allreduce.resid(which, residual, scratch.rowsq, nb)
            # tiles the kernel wrote: its world (a one-rank timing handle in
            # scripts/config5_projection.py has world 1 under a TP-8 shard)
            scratch.stat_tiles = self._allreduce.world * nb
            return
        import torch.distributed as dist
        p = partial.float()
        dist.all_reduce(p, group=self.group)
        residual.copy_((residual.float() + p).to(torch.bfloat16))
        scratch.seed_stats(residual, sums=False)


class LlamaWeights:
    def __init__(self, cfg: LlamaConfig, device, dtype=torch.bfloat16, seed: int = 0,
                 tp: TPGroup | None = None, compact: bool = False):
        tp = tp or TPGroup()
        self.cfg, self.tp = cfg, tp
        # compact: ONE copy of every projection, in the fused decode layout
        # (prefill then runs through the fused GEMMs in <= 64-token chunks).
        # Llama-3-70B bf16 (141 GB) fits one 288 GB MI355X this way, and a
        # TP=8 shard (17.6 GB) fits eight ranks sharing one GPU; the default
        # keeps row-major copies for hipBLASLt prefill as well.
        self.compact = compact
        assert cfg.n_heads % tp.world == 0 and cfg.n_kv_heads % tp.world == 0
        assert cfg.ffn_dim % tp.world == 0 and cfg.vocab_size % tp.world == 0
        self.h = cfg.n_heads // tp.world
        self.hkv = cfg.n_kv_heads // tp.world
        self.f = cfg.ffn_dim // tp.world
        self.v = cfg.vocab_size // tp.world
        d, D, r = cfg.d_model, cfg.head_dim, tp.rank
        H, Hkv, F, V = cfg.n_heads, cfg.n_kv_heads, cfg.ffn_dim, cfg.vocab_size

        # Counter-based init (ops.init_normal): every tensor is a function of
        # (seed, layer, name, global index), so a TP rank generates exactly its
        # Megatron slice of the SAME model the single-GPU engine builds -
        # column-parallel q/k/v, gate/up and vocab rows, row-parallel o / down
        # columns - and TP=N is comparable token for token with TP=1.
        def rnd(key, rows, cols, *, ld=None, row0=0, col0=0):
            return ops.init_normal(rows, cols, seed=seed, key=key, ld=ld, row0=row0, col0=col0,
                                   device=device).to(dtype)

        def ones(n):
            return torch.ones(n, dtype=dtype, device=device)

        # the embedding table is replicated on every TP rank (2.1 GB for the
        # 128k x 8192 table - cheap in 288 GB of HBM), so a decode step's
        # embedding needs no all-reduce; the lm_head stays vocab-parallel
        self.embed = rnd(("embed",), V, d)
        self.layers = []
        if compact:
            self.decode_layers = []
        for li in range(cfg.n_layers):
            L = {
                "attn_norm": ones(d),
                "wqkv": torch.cat([rnd((li, "q"), self.h * D, d, row0=r * self.h * D),
                                   rnd((li, "k"), self.hkv * D, d, row0=r * self.hkv * D),
                                   rnd((li, "v"), self.hkv * D, d, row0=r * self.hkv * D)]),
                "wo": rnd((li, "o"), d, self.h * D, ld=H * D, col0=r * self.h * D),
                "mlp_norm": ones(d),
                "w_gate_up": torch.cat([rnd((li, "gate"), self.f, d, row0=r * self.f),
                                        rnd((li, "up"), self.f, d, row0=r * self.f)]),
                "w_down": rnd((li, "down"), d, self.f, ld=F, col0=r * self.f),
            }
            if compact:   # convert layer by layer: peak = one layer's row-major copy
                self.decode_layers.append(self._compact_layer(L))
                L = {"attn_norm": L["attn_norm"], "mlp_norm": L["mlp_norm"]}
            self.layers.append(L)
        self.final_norm = ones(d)
        vs = slice(r * self.v, (r + 1) * self.v)
        self.lm_head = self.embed[vs] if cfg.tie_embeddings else \
            rnd(("lm_head",), self.v, d, row0=r * self.v)
        self.cos_sin = rope_cos_sin(D, cfg.max_positions, cfg.rope_theta, device=device,
                                    scaling=cfg.rope_scaling)
        self._finalize()

    def _compact_layer(self, L: dict) -> dict:
        from ..ops import reference as _ref
        dev = L["wqkv"].device
        pq = _ref.perm_rope_qkv(self.h, self.hkv, self.cfg.head_dim).to(dev)
        pg = _ref.perm_gate_up(self.f).to(dev)
        return {"wqkv_f": ops.shuffle_weight(ops.fold_norm(L["wqkv"], L["attn_norm"])[pq].contiguous()),
                "w_gate_up_f": ops.shuffle_weight(
                    ops.fold_norm(L["w_gate_up"], L["mlp_norm"])[pg].contiguous()),
                "wo": ops.shuffle_weight(L["wo"]), "w_down": ops.shuffle_weight(L["w_down"])}

    def _finalize(self) -> None:
        """Derived decode copies + split-K tuning (after the base tensors exist)."""
        if getattr(self, "compact", False):
            self.lm_head_p = self._shuffle_lm_head()
            if not self.cfg.tie_embeddings:
                del self.lm_head          # only the shuffled copy is read
            self.fused = True
            if self.embed.device.type == "cuda":
                ops.tune_skinny_splits(self.lm_head_p)
                self._tune_fused()
            return
        # decode copies in MFMA-fragment order for the weight-streaming skinny GEMM
        # (prefill keeps the row-major copies for hipBLASLt; 288 GB of HBM makes
        # the duplicate affordable and each path gets its ideal layout)
        self.decode_layers = [{k: ops.shuffle_weight(L[k])
                               for k in ("wqkv", "wo", "w_gate_up", "w_down")}
                              for L in self.layers]
        self.lm_head_p = self._shuffle_lm_head()
        self._add_fused_copies()
        if self.embed.device.type == "cuda":
            for k in ("wqkv", "wo", "w_gate_up", "w_down"):
                ops.tune_skinny_splits(self.decode_layers[0][k])
            ops.tune_skinny_splits(self.lm_head_p)

    def _shuffle_lm_head(self):
        """Decode copy of the (vocab-shard) lm_head, rows zero-padded to a
        multiple of 64 (the skinny GEMM's 64-row tiles at Mpad 64/128; a TP=8
        Llama-3 shard has 16032 rows); ``LlamaModel`` slices the padding off."""
        w = self.lm_head
        pad = -w.shape[0] % 64
        if pad:
            w = torch.cat([w, torch.zeros(pad, w.shape[1], dtype=w.dtype, device=w.device)])
        return ops.shuffle_weight(w.contiguous())

    @classmethod
    def from_tensors(cls, cfg: LlamaConfig, device, *, embed, layers: list[dict], final_norm,
                     lm_head=None, tp: TPGroup | None = None) -> "LlamaWeights":
        """Weights from explicit tensors (checkpoint loaders): ``layers`` hold
        attn_norm / wqkv (q|k|v rows) / wo / mlp_norm / w_gate_up (gate|up rows)
        / w_down. Unsharded tensors; ``tp`` > 1 shards them (Megatron split)."""
        self = cls.__new__(cls)
        self.cfg, self.tp = cfg, TPGroup()
        self.h, self.hkv, self.f, self.v = cfg.n_heads, cfg.n_kv_heads, cfg.ffn_dim, cfg.vocab_size
        self.embed = embed
        self.layers = layers
        self.final_norm = final_norm
        self.lm_head = self.embed if (cfg.tie_embeddings or lm_head is None) else lm_head
        self.cos_sin = rope_cos_sin(cfg.head_dim, cfg.max_positions, cfg.rope_theta, device=device,
                                    scaling=cfg.rope_scaling)
        if tp is not None and tp.world > 1:
            self.decode_layers, self.lm_head_p = [], None
            return cls.shard(self, tp)
        self._finalize()
        return self

    def _add_fused_copies(self) -> None:
        """Row-permuted decode copies for the fused-epilogue GEMMs (RoPE pairs /
        gate-up pairs share a 32-row tile); TP ranks permute their own slices."""
        self.fused = True
        from ..ops import reference as _ref
        pq = _ref.perm_rope_qkv(self.h, self.hkv, self.cfg.head_dim).to(self.embed.device)
        pg = _ref.perm_gate_up(self.f).to(self.embed.device)
        for L, P in zip(self.layers, self.decode_layers):
            P["wqkv_f"] = ops.shuffle_weight(ops.fold_norm(L["wqkv"], L["attn_norm"])[pq].contiguous())
            P["w_gate_up_f"] = ops.shuffle_weight(
                ops.fold_norm(L["w_gate_up"], L["mlp_norm"])[pg].contiguous())
        if self.embed.device.type == "cuda":
            self._tune_fused()

    def _tune_fused(self) -> None:
        """Measure the split-K of each fused decode GEMM shape (layer-0 weights)."""
        P, D = self.decode_layers[0], self.cfg.head_dim
        pf = bool(getattr(self, "compact", False))
        # TP ranks with prologue launches: qkv / o / gate|up tuned over the
        # layouts those launches run (same order with or without them)
        pc = self.tp.world > 1 and ops.TP_PROLOGUE
        ops.tune_fused(P["wqkv_f"], "rope", norm="rms", heads=(self.h, self.hkv, D),
                       cos_sin=self.cos_sin, prefill=pf, pro_compat=pc)
        ops.tune_fused(P["w_gate_up_f"], "silu", norm="rms", prefill=pf, pro_compat=pc)
        # TP: the row-parallel projections emit bf16 partials ("act" epilogue)
        # that the all-reduce kernel adds to the residual stream
        mode = "resid" if self.tp.world == 1 else "act"
        ops.tune_fused(P["wo"], mode, prefill=pf, pro_compat=pc)
        ops.tune_fused(P["w_down"], mode, prefill=pf)

    @classmethod
    def shard(cls, full: "LlamaWeights", tp: TPGroup) -> "LlamaWeights":
        """Tensor-parallel shard ``tp.rank`` of an unsharded model (Megatron
        split: column-parallel QKV / gate|up / vocab, row-parallel O / down), so
        a TP group computes exactly what the single-GPU model computes."""
        cfg = full.cfg
        assert full.tp.world == 1
        self = cls.__new__(cls)
        self.cfg, self.tp = cfg, tp
        self.h, self.hkv = cfg.n_heads // tp.world, cfg.n_kv_heads // tp.world
        self.f, self.v = cfg.ffn_dim // tp.world, cfg.vocab_size // tp.world
        r, D = tp.rank, cfg.head_dim
        H, Hkv, F = cfg.n_heads, cfg.n_kv_heads, cfg.ffn_dim
        qs, ks = slice(r * self.h * D, (r + 1) * self.h * D), slice(r * self.hkv * D, (r + 1) * self.hkv * D)
        fs, vs = slice(r * self.f, (r + 1) * self.f), slice(r * self.v, (r + 1) * self.v)
        self.compact = False
        self.embed = full.embed          # replicated (see __init__)
        self.layers = []
        for L in full.layers:
            w = L["wqkv"]
            q, k, v = w[: H * D], w[H * D:(H + Hkv) * D], w[(H + Hkv) * D:]
            gu = L["w_gate_up"]
            self.layers.append({
                "attn_norm": L["attn_norm"],
                "wqkv": torch.cat([q[qs], k[ks], v[ks]]).contiguous(),
                "wo": L["wo"][:, qs].contiguous(),
                "mlp_norm": L["mlp_norm"],
                "w_gate_up": torch.cat([gu[:F][fs], gu[F:][fs]]).contiguous(),
                "w_down": L["w_down"][:, fs].contiguous()})
        self.final_norm = full.final_norm
        self.lm_head = (full.embed if cfg.tie_embeddings else full.lm_head)[vs].contiguous()
        self.cos_sin = full.cos_sin
        self._finalize()
        return self

    def nbytes(self) -> int:
        n = self.embed.numel() + (0 if self.cfg.tie_embeddings else self.lm_head.numel())
        for L in self.layers:
            n += sum(t.numel() for t in L.values())
        return n * 2


# prompt passes on the hand-written GEMMs (ops.proj: split-K tiled / weight-
# streaming MFMA kernels with fused SwiGLU / residual epilogues); 0: hipBLASLt
# (measured: 19.23 / 19.30 vs 19.15 / 18.99 utt/s, docs/PERF.md "Round 4")
PREFILL_HW = os.environ.get("LOQA_PREFILL_HW", "1") != "0"



def L0_KEYS(w) -> set:
    return set(w.layers[0]) if w.layers else set()


class LlamaModel:
    def __init__(self, w: LlamaWeights):
        self.w = w
        self.cfg = w.cfg

    def embed(self, tokens: torch.Tensor) -> torch.Tensor:
        tp = self.w.tp
        if tp.world == 1 or self.w.embed.shape[0] == self.cfg.vocab_size:   # replicated table
            return torch.nn.functional.embedding(tokens.long(), self.w.embed)
        lo = tp.rank * self.w.v
        local = tokens.long() - lo
        inr = (local >= 0) & (local < self.w.v)
        x = torch.nn.functional.embedding(local.clamp(0, self.w.v - 1), self.w.embed)
        x = x * inr[:, None].to(x.dtype)
        return tp.all_reduce_(x)

    def forward(self, meta: StepMeta, k_cache: torch.Tensor, v_cache: torch.Tensor,
                attn_ws: ops.AttnWorkspace | None = None) -> torch.Tensor:
        """Runs all layers; returns final-normed hidden states of ``logit_idx`` rows
        [B, d]. k_cache/v_cache: [L, n_blocks, Hkv, BLK, D]."""
        cfg, w, tp = self.cfg, self.w, self.w.tp
        H, Hkv, D = w.h, w.hkv, cfg.head_dim
        x = self.embed(meta.tokens)
        residual = x
        h = ops.rmsnorm(x, w.layers[0]["attn_norm"], cfg.norm_eps)
        split_keys = 256
        num_splits = max(1, (meta.max_ctx + split_keys - 1) // split_keys)
        if (PREFILL_HW and x.is_cuda and not meta.decode
                and not getattr(w, "compact", False) and "wqkv" in L0_KEYS(w)):
            return self._forward_prefill_hw(meta, k_cache, v_cache, attn_ws, x, h)
        for li, L in enumerate(w.layers):
            if li > 0:
                h = ops.rmsnorm(mlp_out, L["attn_norm"], cfg.norm_eps, residual=residual)
            qkv = ops.linear(h, L["wqkv"])
            ops.rope_kv_append(qkv, meta.positions, w.cos_sin, k_cache[li], v_cache[li], meta.slots,
                               H, Hkv, D)
            if meta.split is not None:
                attn = self._prompt_attention(meta, qkv, k_cache[li], v_cache[li], attn_ws)
            else:
                attn = ops.attention(qkv, k_cache[li], v_cache[li], meta.cu_q, n_heads=H, n_kv=Hkv,
                                     head_dim=D, causal=True, max_q=meta.max_q,
                                     ctx_lens=meta.ctx_lens, block_tables=meta.block_tables,
                                     grouped=meta.decode, split_keys=split_keys,
                                     num_splits=num_splits if meta.decode else 1,
                                     workspace=attn_ws, max_k=meta.max_ctx)
            o = tp.all_reduce_(ops.linear(attn, L["wo"]))
            h = ops.rmsnorm(o, L["mlp_norm"], cfg.norm_eps, residual=residual)
            gu = ops.linear(h, L["w_gate_up"])
            mlp_out = tp.all_reduce_(ops.linear(ops.silu_mul(gu), L["w_down"]))
        sel_res = residual.index_select(0, meta.logit_idx)
        sel_mlp = mlp_out.index_select(0, meta.logit_idx)
        return ops.rmsnorm(sel_mlp.contiguous(), w.final_norm, cfg.norm_eps,
                           residual=sel_res.contiguous())

    def _prompt_attention(self, meta: StepMeta, qkv: torch.Tensor, kc: torch.Tensor,
                          vc: torch.Tensor, attn_ws) -> torch.Tensor:
        """Attention of a prompt (or mixed) pass. A mixed pass (``meta.split``)
        runs its leading live-decoder rows on the grouped split-key decode
        kernel - each kv head's cache read once for its G q heads - and the
        prompt chunk rows on the flash prefill kernel, which would otherwise
        take a 128-row query tile per decoder row and head and re-read that
        sequence's whole cache per q head (G = 4 times)."""
        w = self.w
        H, Hkv, D = w.h, w.hkv, self.cfg.head_dim
        if meta.split is None:
            return ops.attention(qkv, kc, vc, meta.cu_q, n_heads=H, n_kv=Hkv, head_dim=D,
                                 causal=True, max_q=meta.max_q, ctx_lens=meta.ctx_lens,
                                 block_tables=meta.block_tables, grouped=False, split_keys=256,
                                 num_splits=1, workspace=attn_ws, max_k=meta.max_ctx)
        nd, rd, dq, dctx, cu_tail = meta.split
        attn = torch.empty(qkv.shape[0], H * D, dtype=torch.bfloat16, device=qkv.device)
        ns, sk = ops.decode_attn_splits(dctx, nd * Hkv, 128, getattr(w, "max_wgs", None))
        ops.attention(qkv[:rd], kc, vc, meta.cu_q[:nd + 1], n_heads=H, n_kv=Hkv, head_dim=D,
                      causal=True, max_q=dq, ctx_lens=meta.ctx_lens[:nd],
                      block_tables=meta.block_tables[:nd], grouped=True, split_keys=sk,
                      num_splits=ns, workspace=attn_ws, out=attn[:rd], max_k=dctx)
        ops.attention(qkv[rd:], kc, vc, cu_tail, n_heads=H, n_kv=Hkv, head_dim=D, causal=True,
                      max_q=meta.max_q, ctx_lens=meta.ctx_lens[nd:],
                      block_tables=meta.block_tables[nd:], grouped=False, split_keys=256,
                      num_splits=1, workspace=attn_ws, out=attn[rd:], max_k=meta.max_ctx)
        return attn

    def _forward_prefill_hw(self, meta: StepMeta, k_cache, v_cache, attn_ws, x, h
                            ) -> torch.Tensor:
        """Prompt pass on the hand-written GEMMs (``ops.proj``: per shape the
        measured faster of the split-K tiled GEMM, whose K chunks are summed
        in-launch, and the row-resident weight-streaming GEMM; tensor parallel:
        the same GEMMs on the rank's shards, the row-parallel o / down partials
        summed by the custom all-reduce - no hipBLASLt on any rank): per layer qkv
        (bf16) -> RoPE + KV append -> flash attention -> o added straight into
        the residual stream (one rounding) -> RMSNorm -> gate|up with the
        SwiGLU epilogue -> down added into the residual -> the next layer's
        RMSNorm. No hipBLASLt call, no f32 slab written or re-read. (o / down
        as prefill-GEMM f32 slabs summed by the next norm is 9% faster alone,
        7.73 vs 8.46 ms per 318-token pass, but ~1% slower beside the
        decoders: docs/PERF.md "Round 4".)"""
        cfg, w, tp = self.cfg, self.w, self.w.tp
        H, Hkv, D = w.h, w.hkv, cfg.head_dim
        residual = x.contiguous()
        dn = None
        for li, L in enumerate(w.layers):
            if li > 0:
                # TP: the previous down partials (all-reduced) join the residual here
                h = (ops.rmsnorm(residual, L["attn_norm"], cfg.norm_eps) if dn is None else
                     ops.rmsnorm(dn, L["attn_norm"], cfg.norm_eps, residual=residual))
            qkv = ops.proj(h, L["wqkv"])
            ops.rope_kv_append(qkv, meta.positions, w.cos_sin, k_cache[li], v_cache[li], meta.slots,
                               H, Hkv, D)
            attn = self._prompt_attention(meta, qkv, k_cache[li], v_cache[li], attn_ws)
            if tp.world == 1:
                ops.proj(attn, L["wo"], epi="resid", residual=residual)
                hn = ops.rmsnorm(residual, L["mlp_norm"], cfg.norm_eps)
            else:
                # row-parallel o: this rank's partial on the hand-written GEMM,
                # the custom all-reduce (two-shot over xGMI at prompt sizes),
                # then residual add + RMSNorm in one kernel
                o = ops.proj(attn, L["wo"])
                tp.all_reduce_(o)
                hn = ops.rmsnorm(o, L["mlp_norm"], cfg.norm_eps, residual=residual)
            a = ops.proj(hn, L["w_gate_up"], epi="swiglu")
            if tp.world == 1:
                ops.proj(a, L["w_down"], epi="resid", residual=residual)
            else:
                dn = ops.proj(a, L["w_down"])
                tp.all_reduce_(dn)
        if dn is not None:
            residual.add_(dn)          # one bf16 rounding, as the norm's residual add
        return ops.rmsnorm(residual, w.final_norm, cfg.norm_eps, row_idx=meta.logit_idx)

    def _ones(self, x: torch.Tensor) -> torch.Tensor:
        t = getattr(self, "_ones_d", None)
        if t is None or t.device != x.device:
            t = self._ones_d = torch.ones(self.cfg.d_model, dtype=x.dtype, device=x.device)
        return t

    def forward_decode(self, meta: StepMeta, k_cache: torch.Tensor, v_cache: torch.Tensor,
                       attn_ws: ops.AttnWorkspace | None, split_keys: int = 128) -> torch.Tensor:
        """Decode / jump-forward step for <= 128 padded tokens. Every projection is
        the weight-streaming skinny MFMA GEMM emitting split-K f32 slabs that the
        following fused kernel reduces (rmsnorm+residual, RoPE+KV append, SwiGLU).
        ``meta.tokens`` has Mpad rows; ``meta.logit_idx`` has >= 16 rows.
        Returns f32 logits [len(logit_idx), V/tp]."""
        cfg, w, tp = self.cfg, self.w, self.w.tp
        H, Hkv, D = w.h, w.hkv, cfg.head_dim
        tp_splits = 1 if tp.world > 1 else None
        x = self.embed(meta.tokens)
        residual = x.contiguous()
        h = ops.rmsnorm(residual, w.layers[0]["attn_norm"], cfg.norm_eps)
        num_splits = max(1, (meta.max_ctx + split_keys - 1) // split_keys)
        down = None
        for li, L in enumerate(w.layers):
            P = w.decode_layers[li]
            if li > 0:
                h = ops.slab_rmsnorm(down, residual, L["attn_norm"], cfg.norm_eps)
            qkv = ops.skinny_gemm(h, P["wqkv"])
            q = ops.slab_rope_append(qkv, meta.positions, w.cos_sin, k_cache[li], v_cache[li],
                                     meta.slots, H, Hkv, D)
            attn = ops.attention(q, k_cache[li], v_cache[li], meta.cu_q, n_heads=H, n_kv=Hkv,
                                 head_dim=D, causal=True, max_q=meta.max_q, ctx_lens=meta.ctx_lens,
                                 block_tables=meta.block_tables, grouped=True,
                                 split_keys=split_keys, num_splits=num_splits, workspace=attn_ws,
                                 max_k=meta.max_ctx)
            o = ops.skinny_gemm(attn, P["wo"], tp_splits)
            tp.all_reduce_(o)
            h = ops.slab_rmsnorm(o, residual, L["mlp_norm"], cfg.norm_eps)
            gu = ops.skinny_gemm(h, P["w_gate_up"])
            a = ops.slab_silu_mul(gu)
            down = ops.skinny_gemm(a, P["w_down"], tp_splits)
            tp.all_reduce_(down)
        hf = ops.slab_rmsnorm(down, residual, w.final_norm, cfg.norm_eps, row_idx=meta.logit_idx,
                              write_residual=False)
        return ops.skinny_gemm(hf, w.lm_head_p, 1,
                               max_wgs=getattr(w, "max_wgs", ops.MAX_DECODE_WGS))[0][:, :w.v]

    def forward_decode_fused(self, meta: StepMeta, k_cache: torch.Tensor, v_cache: torch.Tensor,
                             attn_ws: ops.AttnWorkspace | None, scratch: ops.FusedScratch,
                             split_keys: int = 128) -> torch.Tensor:
        """Decode step with the fused-epilogue GEMMs (5 launches per layer):
        qkv (RMSNorm prologue, RoPE + KV append epilogue) -> attention ->
        o (residual + row sum-of-squares epilogue) -> gate|up (RMSNorm prologue,
        SwiGLU epilogue) -> down (residual + row sum-of-squares); Mpad 16 / 32 /
        64. Same numerics as ``forward_decode``. Tensor parallel:
        o and down emit bf16 partials and the residual all-reduce kernel adds
        them (7 launches per layer); the logits are this rank's vocab slice."""
        cfg, w, tp = self.cfg, self.w, self.w.tp
        H, Hkv, D, d = w.h, w.hkv, cfg.head_dim, cfg.d_model
        Mpad = meta.tokens.numel()
        # embedding + layer 0's RMSNorm row scale (one partial sum of squares per
        # row) in one launch (TP ranks hold the whole table)
        if ops.FUSED_EMBED and w.embed.shape[0] == cfg.vocab_size and meta.tokens.dtype == torch.int32:
            residual = ops.embed_stats(meta.tokens, w.embed, scratch)
        else:
            residual = self.embed(meta.tokens).contiguous()
            scratch.seed_stats(residual, sums=False)
        num_splits, split_keys = ops.decode_attn_splits(meta.max_ctx, meta.ctx_lens.numel() * Hkv,
                                                        split_keys, getattr(w, "max_wgs", None))
        q = torch.empty(Mpad, H * D, dtype=torch.bfloat16, device=residual.device)
        # chunked prefill through this path (compact weights) can exceed the
        # grouped kernels' row limit: plain varlen flash attention then
        grouped = (H // Hkv) * meta.max_q <= 128
        # decode rows (the split-key kernel's <= 32 query rows per kv head): qkv
        # and attention through skinny_fused(attn=)
        dec_attn = (H // Hkv) * meta.max_q <= 32 and attn_ws is not None
        ao = torch.empty(Mpad, H * D, dtype=torch.bfloat16, device=residual.device) if dec_attn else None
        car = tp.car if tp.world > 1 else None
        if (car is not None and dec_attn and ops.TP_PROLOGUE and Mpad in (16, 32)
                and residual.is_cuda and D == 128):
            return self._decode_fused_tp_prologue(meta, k_cache, v_cache, attn_ws, scratch, residual, q,
                                                  ao, num_splits, split_keys, car)
        for li, L in enumerate(w.layers):
            P = w.decode_layers[li]
            if dec_attn:
                attn = ops.skinny_fused(
                    residual, P["wqkv_f"], "rope", scratch, norm=True, eps=cfg.norm_eps,
                    positions=meta.positions, cos_sin=w.cos_sin, q_out=q, k_cache=k_cache[li],
                    v_cache=v_cache[li], slots=meta.slots, n_heads=H, n_kv=Hkv, head_dim=D,
                    attn=dict(cu_q=meta.cu_q, ctx_lens=meta.ctx_lens,
                              block_tables=meta.block_tables, max_q=meta.max_q,
                              split_keys=split_keys, num_splits=num_splits, workspace=attn_ws,
                              max_k=meta.max_ctx, out=ao))
            else:
                ops.skinny_fused(residual, P["wqkv_f"], "rope", scratch, norm=True,
                                 eps=cfg.norm_eps,
                                 positions=meta.positions, cos_sin=w.cos_sin, q_out=q,
                                 k_cache=k_cache[li], v_cache=v_cache[li], slots=meta.slots,
                                 n_heads=H, n_kv=Hkv, head_dim=D)
                attn = ops.attention(q, k_cache[li], v_cache[li], meta.cu_q, n_heads=H, n_kv=Hkv,
                                     head_dim=D, causal=True, max_q=meta.max_q,
                                     ctx_lens=meta.ctx_lens, block_tables=meta.block_tables,
                                     grouped=grouped, split_keys=split_keys,
                                     num_splits=num_splits if grouped else 1,
                                     workspace=attn_ws, max_k=meta.max_ctx)
            if tp.world == 1:
                ops.skinny_fused(attn, P["wo"], "resid", scratch, residual=residual)
            else:
                # row-parallel o: f32 partial into the all-reduce input buffer,
                # then ONE kernel sums the ranks into the residual + row stats
                po = tp.partial_out(0, Mpad, d, residual.device)
                ops.skinny_fused(attn, P["wo"], "act", scratch, out=po, act="f32")
                tp.resid_epilogue(0, po, residual, scratch)
            a = ops.skinny_fused(residual, P["w_gate_up_f"], "silu", scratch, norm=True,
                                 eps=cfg.norm_eps)
            if tp.world == 1:
                ops.skinny_fused(a, P["w_down"], "resid", scratch, residual=residual)
            else:
                pd = tp.partial_out(1, Mpad, d, residual.device)
                ops.skinny_fused(a, P["w_down"], "act", scratch, out=pd, act="f32")
                tp.resid_epilogue(1, pd, residual, scratch)
        if ops.FUSED_EMBED:
            hf = ops.rmsnorm(residual, w.final_norm, cfg.norm_eps, row_idx=meta.logit_idx)
        else:
            hf = ops.rmsnorm(residual.index_select(0, meta.logit_idx), w.final_norm, cfg.norm_eps)
        return ops.skinny_gemm(hf, w.lm_head_p, 1,
                               max_wgs=getattr(w, "max_wgs", ops.MAX_DECODE_WGS))[0][:, :w.v]

    def _decode_fused_tp_prologue(self, meta, k_cache, v_cache, attn_ws, scratch, residual, q, ao,
                                  num_splits, split_keys, car) -> torch.Tensor:
        """The tensor-parallel decode step with every latency-bound step run as
        the prologue of the GEMM that consumes it (ops.skinny_fused
        ``prologue``; gemm_skinny.hip PRO): 4 launches per layer instead of 7 -
        qkv (+ the previous layer's down all-reduce) -> o (+ the decode
        attention) -> gate|up (+ the o all-reduce) -> down. Each GEMM's weight
        stream starts while its prologue's flag exchanges and KV reads are in
        flight; numerics are those of the 7-launch step (same arithmetic, same
        order)."""
        cfg, w, tp = self.cfg, self.w, self.w.tp
        H, Hkv, D, d = w.h, w.hkv, cfg.head_dim, cfg.d_model
        Mpad = meta.tokens.numel()
        nb = car.resid_blocks(d)
        pw = car.prologue_wgs(d)
        att = dict(kind="attn", q=q, cu_q=meta.cu_q, ctx_lens=meta.ctx_lens,
                   block_tables=meta.block_tables, n_heads=H, n_kv=Hkv, max_q=meta.max_q,
                   split_keys=split_keys, num_splits=num_splits, workspace=attn_ws,
                   max_k=meta.max_ctx, pro_wgs=pw)
        for li in range(len(w.layers)):
            P = w.decode_layers[li]
            pro = None
            if li > 0:        # the previous layer's down all-reduce -> this qkv
                pro = dict(kind="car", car=car, which=1, nblk=nb, pro_wgs=pw)
                scratch.stat_tiles = car.world * nb
            ops.skinny_fused(residual, P["wqkv_f"], "rope", scratch, norm=True, eps=cfg.norm_eps,
                             positions=meta.positions, cos_sin=w.cos_sin, q_out=q,
                             k_cache=k_cache[li], v_cache=v_cache[li], slots=meta.slots,
                             n_heads=H, n_kv=Hkv, head_dim=D, prologue=pro)
            po = tp.partial_out(0, Mpad, d, residual.device)
            ops.skinny_fused(ao, P["wo"], "act", scratch, out=po, act="f32",
                             prologue=dict(att, k_cache=k_cache[li], v_cache=v_cache[li]))
            scratch.stat_tiles = car.world * nb
            a = ops.skinny_fused(residual, P["w_gate_up_f"], "silu", scratch, norm=True,
                                 eps=cfg.norm_eps,
                                 prologue=dict(kind="car", car=car, which=0, nblk=nb, pro_wgs=pw))
            pd = tp.partial_out(1, Mpad, d, residual.device)
            ops.skinny_fused(a, P["w_down"], "act", scratch, out=pd, act="f32")
        tp.resid_epilogue(1, pd, residual, scratch)
        if ops.FUSED_EMBED:
            hf = ops.rmsnorm(residual, w.final_norm, cfg.norm_eps, row_idx=meta.logit_idx)
        else:
            hf = ops.rmsnorm(residual.index_select(0, meta.logit_idx), w.final_norm, cfg.norm_eps)
        return ops.skinny_gemm(hf, w.lm_head_p, 1,
                               max_wgs=getattr(w, "max_wgs", ops.MAX_DECODE_WGS))[0][:, :w.v]

    def logits(self, hidden: torch.Tensor) -> torch.Tensor:
        """Local vocab shard logits [B, V/tp]. On the GPU the prompt pass's few
        sampling rows go through the decode steps' weight-streaming lm_head
        (pre-shuffled copy, rows padded to 16; f32 logits), not hipBLASLt."""
        w = self.w
        B = hidden.shape[0]
        if (hidden.is_cuda and getattr(w, "lm_head_p", None) is not None
                and B <= ops.MPADS[-1]):
            Mpad = ops.mpad_for(B)
            x = hidden
            if Mpad != B:
                x = torch.zeros(Mpad, hidden.shape[1], dtype=hidden.dtype, device=hidden.device)
                x[:B] = hidden
            return ops.skinny_gemm(x.contiguous(), w.lm_head_p, 1,
                                   max_wgs=getattr(w, "max_wgs", ops.MAX_DECODE_WGS))[0][:B, :w.v]
        return ops.linear(hidden, w.lm_head)
