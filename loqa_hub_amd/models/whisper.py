"""Whisper encoder/decoder (tiny/base/small/large-v3) for on-GPU STT, replacing the
reference's ``POST {STT_URL}/v1/audio/transcriptions`` (``stt_client.go:157``,
``model=tiny``, temperature 0 = greedy).

Execution plan per batch of utterances (one GPU):
  log-mel (f32-MFMA STFT kernel) -> conv stem as im2col + GEMM with fused
  bias+GELU(+sinusoidal position) epilogue -> L pre-LN encoder blocks (fused
  QKV GEMM, non-causal flash attention on the contiguous QKV output, fused
  residual+layernorm) -> cross-attention K/V for every decoder layer computed
  once -> greedy decode with a paged self-attention cache and split-K
  cross-attention over the 1500 encoder frames.
"""
from __future__ import annotations

import math
import os

import numpy as np
import torch

from .. import ops
from ..ops.reference import MelConstants
from .configs import WhisperConfig


def sinusoids(length: int, channels: int, max_timescale: float = 10000.0) -> torch.Tensor:
    lt = math.log(max_timescale) / (channels // 2 - 1)
    inv = torch.exp(-lt * torch.arange(channels // 2, dtype=torch.float64))
    t = torch.arange(length, dtype=torch.float64)[:, None] * inv[None, :]
    return torch.cat([t.sin(), t.cos()], dim=1).float()


DEC_PROJ = ("wqkv", "wo", "xq", "xo", "fc1", "fc2")

# Measured choices (docs/PERF.md), module constants so tests can flip them:
# split-K of the encoder o projection on the prefill GEMM (0: hipBLASLt)
ENC_O_SPLITS = 2
# conv stem (implicit-im2col conv1d with bias + GELU (+ positions) fused) and
# the fc2 projection (split-K slabs summed by the next LayerNorm) on the
# LDS-tiled MFMA GEMM (csrc/kernels/gemm_tile.hip); False: im2col + hipBLASLt
ENC_TILE = True
ENC_FC2_SPLITS = 4
# cross-attention K|V of ALL decoder layers as one tiled-GEMM launch over the
# layer-concatenated weights (False: one hipBLASLt GEMM per layer)
XKV_TILE = True
# every encoder projection on the hand-written GEMMs (ops.proj: split-K tiled;
# 19.26 / 19.10 vs 19.11 / 19.11 utt/s with qkv / fc1 on hipBLASLt,
# docs/PERF.md "Round 4"); 0: hipBLASLt qkv / fc1, prefill GEMM v2 o
ENC_SK = int(os.environ.get("LOQA_ENC_SK", "1"))


class WhisperWeights:
    def __init__(self, cfg: WhisperConfig, device, dtype=torch.bfloat16, seed: int = 0):
        self.cfg = cfg
        d, f, M = cfg.d_model, cfg.ffn_dim, cfg.n_mels
        g = torch.Generator(device=device)
        g.manual_seed(seed * 7919 + 3)

        def rnd(*shape, std=0.02):
            t = torch.empty(*shape, dtype=dtype, device=device)
            t.normal_(0.0, std, generator=g)
            return t

        def zeros(*shape):
            return torch.zeros(*shape, dtype=dtype, device=device)

        def ones(n):
            return torch.ones(n, dtype=dtype, device=device)

        self.conv1_w = rnd(d, M * 3)          # [Cout, Cin*3] (torch conv weight flattened)
        self.conv1_b = zeros(d)
        self.conv2_w = rnd(d, d * 3)
        self.conv2_b = zeros(d)
        self.pos_enc = sinusoids(cfg.n_audio_ctx, d).to(device=device, dtype=dtype)
        self.enc = []
        for _ in range(cfg.enc_layers):
            self.enc.append(self._block(rnd, zeros, ones, d, f, cross=False))
        self.enc_ln_w, self.enc_ln_b = ones(d), zeros(d)
        self.tok_embed = rnd(cfg.vocab_size, d)
        self.dec_pos = rnd(cfg.n_text_ctx, d, std=0.01)
        self.dec = []
        for _ in range(cfg.dec_layers):
            self.dec.append(self._block(rnd, zeros, ones, d, f, cross=True))
        self.dec_ln_w, self.dec_ln_b = ones(d), zeros(d)
        self._finalize()

    def _finalize(self) -> None:
        """Derived decode copies + split-K tuning (after the base tensors exist)."""
        cfg, d = self.cfg, self.cfg.d_model
        device, dtype = self.tok_embed.device, self.tok_embed.dtype
        # decode-path copies in MFMA fragment order for the weight-streaming
        # skinny GEMM; the vocab is zero-padded to a multiple of 32 rows
        self.vocab_pad = (cfg.vocab_size + 31) // 32 * 32
        lm = torch.zeros(self.vocab_pad, d, dtype=dtype, device=device)
        lm[: cfg.vocab_size] = self.tok_embed
        self.lm_head_p = ops.shuffle_weight(lm)
        del lm
        self.dec_p = [{k: ops.shuffle_weight(L[k]) for k in DEC_PROJ} for L in self.dec]
        # encoder o projection on the hand-written prefill GEMM (fragment-order
        # copy; 1500-row windows: 17 vs 21.6 us for hipBLASLt at large-v3,
        # profiles/r3_prefill_gemm2_layouts.txt)
        self.enc_wo_p = ([ops.shuffle_weight(L["wo"]) for L in self.enc]
                         if device.type == "cuda" and d % 128 == 0 and ENC_O_SPLITS else None)
        # conv stem weights in the implicit-im2col order (k = tap * Cin + c)
        # and f32 biases for the tiled GEMM's epilogue
        self.conv1_wt = ops.conv_k3_weight(self.conv1_w, cfg.n_mels)
        self.conv2_wt = ops.conv_k3_weight(self.conv2_w, d)
        self.conv1_bf, self.conv2_bf = self.conv1_b.float(), self.conv2_b.float()
        self.enc_fc1_bf = [L["fc1_b"].float() for L in self.enc]
        self.enc_qkv_bf = [L["bqkv"].float() for L in self.enc]
        self.enc_o_bf = [L["bo"].float() for L in self.enc]
        self.enc_fc2_bf = [L["fc2_b"].float() for L in self.enc]
        # the decoder layers' cross K|V weights as ONE [L * 2d, d] matrix (each
        # layer's "xkv" becomes a row-block view of it, no second copy), so the
        # cross K|V of an utterance is one tiled GEMM launch
        self.xkv_all = self.xkv_all_b = None
        if device.type == "cuda" and XKV_TILE and (len(self.dec) * 2 * d) % 256 == 0 and d % 64 == 0:
            self.xkv_all = torch.cat([L["xkv"] for L in self.dec]).contiguous()
            self.xkv_all_b = torch.cat([L["xkv_b"] for L in self.dec]).float()
            for i, L in enumerate(self.dec):
                L["xkv"] = self.xkv_all[i * 2 * d:(i + 1) * 2 * d]
        # fused-epilogue copies: LayerNorm weight folded into qkv / xq / fc1 rows,
        # LayerNorm shift + linear bias folded into one f32 bias, qkv rows in
        # (c, c + D/2) pair order (the epilogue writes q and the paged K/V)
        self.dec_f = [self._fused_layer(L) for L in self.dec]
        if device.type == "cuda":
            for k in DEC_PROJ:
                ops.tune_skinny_splits(self.dec_p[0][k], mpads=(16, 32))
            ops.tune_skinny_splits(self.lm_head_p, mpads=(16, 32))
            F = self.dec_f[0]
            MP = (16, 32, 64)   # a Whisper decoder step never exceeds 64 tokens
            ops.tune_fused(F["qkv"], "rope", heads=(cfg.n_heads, cfg.n_heads, cfg.head_dim), mpads=MP,
                           xl=False)
            ops.tune_fused(F["o"], "resid", mpads=MP, xl=False)
            ops.tune_fused(F["xq"], "act", mpads=MP, xl=False)
            ops.tune_fused(F["fc1"], "act", act="gelu", mpads=MP, xl=False)
            ops.tune_fused(F["fc2"], "resid", mpads=MP, xl=False)

    @classmethod
    def from_tensors(cls, cfg: WhisperConfig, *, conv1_w, conv1_b, conv2_w, conv2_b, pos_enc, enc,
                     enc_ln_w, enc_ln_b, tok_embed, dec_pos, dec, dec_ln_w,
                     dec_ln_b) -> "WhisperWeights":
        """Weights from explicit tensors (checkpoint loaders); block dicts use
        the ``_block`` names (wqkv = q|k|v rows, xkv = k|v rows)."""
        self = cls.__new__(cls)
        self.cfg = cfg
        self.conv1_w, self.conv1_b, self.conv2_w, self.conv2_b = conv1_w, conv1_b, conv2_w, conv2_b
        self.pos_enc, self.enc, self.enc_ln_w, self.enc_ln_b = pos_enc, enc, enc_ln_w, enc_ln_b
        self.tok_embed, self.dec_pos, self.dec = tok_embed, dec_pos, dec
        self.dec_ln_w, self.dec_ln_b = dec_ln_w, dec_ln_b
        self._finalize()
        return self

    def _fused_layer(self, L: dict) -> dict:
        H, D = self.cfg.n_heads, self.cfg.head_dim
        perm = ops.reference.perm_rope_qkv(H, H, D).to(L["wqkv"].device)
        FL = ops.FusedLinear
        return {
            "qkv": FL(L["wqkv"], norm="ln", norm_w=L["ln1_w"], norm_b=L["ln1_b"], bias=L["bqkv"],
                      perm=perm),
            "o": FL(L["wo"], bias=L["bo"]),
            "xq": FL(L["xq"], norm="ln", norm_w=L["lnx_w"], norm_b=L["lnx_b"], bias=L["xq_b"]),
            "xo": FL(L["xo"], bias=L["xo_b"]),
            "fc1": FL(L["fc1"], norm="ln", norm_w=L["ln2_w"], norm_b=L["ln2_b"], bias=L["fc1_b"]),
            "fc2": FL(L["fc2"], bias=L["fc2_b"]),
        }

    @staticmethod
    def _block(rnd, zeros, ones, d, f, cross: bool) -> dict:
        b = {
            "ln1_w": ones(d), "ln1_b": zeros(d),
            "wqkv": rnd(3 * d, d), "bqkv": zeros(3 * d),   # k bias is zero in whisper
            "wo": rnd(d, d), "bo": zeros(d),
            "ln2_w": ones(d), "ln2_b": zeros(d),
            "fc1": rnd(f, d), "fc1_b": zeros(f),
            "fc2": rnd(d, f), "fc2_b": zeros(d),
        }
        if cross:
            b.update({
                "lnx_w": ones(d), "lnx_b": zeros(d),
                "xq": rnd(d, d), "xq_b": zeros(d),
                "xkv": rnd(2 * d, d), "xkv_b": zeros(2 * d),
                "xo": rnd(d, d), "xo_b": zeros(d),
            })
        return b


class WhisperModel:
    def __init__(self, w: WhisperWeights):
        self.w = w
        self.cfg = w.cfg
        self.mel = MelConstants.create(self.cfg.n_mels)

    # ----------------------------------------------------------------- encoder
    def encode(self, audio: torch.Tensor) -> torch.Tensor:
        """audio [B, 480000] f32 (padded 30 s windows) -> encoder states [B*1500, d] bf16."""
        cfg, w = self.cfg, self.w
        B = audio.shape[0]
        d, M = cfg.d_model, cfg.n_mels
        mel = ops.log_mel(audio, self.mel)  # [B, M, 3000] bf16
        frames = mel.shape[-1]
        tile = ENC_TILE and audio.is_cuda and d % 128 == 0 and M % 64 == 0
        if tile:
            # conv1d stem on the tiled MFMA GEMM: the loader gathers the k = 3
            # taps from time-major rows (no column matrix), bias + GELU (+ the
            # sinusoidal positions for conv2) in the epilogue
            mel_t = mel.transpose(1, 2).contiguous().view(B * frames, M)
            x1 = ops.gemm_tile(mel_t, w.conv1_wt, bias=w.conv1_bf, act="gelu", conv=(B, 1), layout=0)
            x = ops.gemm_tile(x1, w.conv2_wt, bias=w.conv2_bf, act="gelu", pos=w.pos_enc,
                              conv=(B, 2), layout=0)
        else:
            cols = ops.im2col_k3(mel, (M * frames, frames, 1), B, M, frames, 1)
            x1 = ops.linear(cols, w.conv1_w)                      # [B*3000, d]
            ops.gelu_bias_(x1, w.conv1_b)
            cols2 = ops.im2col_k3(x1, (frames * d, 1, d), B, d, frames, 2)
            x = ops.linear(cols2, w.conv2_w)                      # [B*1500, d]
            ops.gelu_bias_(x, w.conv2_b, w.pos_enc)               # + positional embedding
        T = cfg.n_audio_ctx
        cu = torch.arange(0, (B + 1) * T, T, dtype=torch.int32, device=audio.device)
        H, D = cfg.n_heads, cfg.head_dim
        if tile and ENC_SK:
            return self._encode_sk(x, cu, T)
        residual = x
        h = ops.layernorm(x, w.enc[0]["ln1_w"], w.enc[0]["ln1_b"], 1e-5)
        delta = None
        part2 = None
        S2 = ENC_FC2_SPLITS if (tile and cfg.ffn_dim % (ENC_FC2_SPLITS * 64) == 0) else 0
        for i, L in enumerate(w.enc):
            if i > 0:
                if part2 is not None:
                    h = ops.slab_layernorm(part2, residual, L["ln1_w"], L["ln1_b"], 1e-5,
                                           bias=w.enc[i - 1]["fc2_b"])
                else:
                    h = ops.layernorm(delta, L["ln1_w"], L["ln1_b"], 1e-5, residual=residual)
            qkv = ops.linear(h, L["wqkv"], L["bqkv"])
            a = ops.attention(qkv, qkv[:, d:], qkv[:, 2 * d:], cu, n_heads=H, n_kv=H, head_dim=D,
                              causal=False, max_q=T, cu_k=cu)
            if getattr(w, "enc_wo_p", None) is not None and (d // 64) % ENC_O_SPLITS == 0:
                part = ops.prefill_gemm2(a, w.enc_wo_p[i], ENC_O_SPLITS, epi="slabs")
                h = ops.slab_layernorm(part, residual, L["ln2_w"], L["ln2_b"], 1e-5, bias=L["bo"])
            else:
                o = ops.linear(a, L["wo"], L["bo"])
                h = ops.layernorm(o, L["ln2_w"], L["ln2_b"], 1e-5, residual=residual)
            m = ops.linear(h, L["fc1"], L["fc1_b"])
            ops.gelu_bias_(m)
            if S2:
                # fc2 as split-K f32 slabs (hipBLASLt's N = 1280 tiles leave
                # most CUs idle at 1500 rows), summed by the next LayerNorm
                part2 = ops.gemm_tile(m, L["fc2"], epi="slabs", splits=S2, layout=0)
            else:
                delta = ops.linear(m, L["fc2"], L["fc2_b"])
        if part2 is not None:
            return ops.slab_layernorm(part2, residual, w.enc_ln_w, w.enc_ln_b, 1e-5,
                                      bias=w.enc[-1]["fc2_b"])
        return ops.layernorm(delta, w.enc_ln_w, w.enc_ln_b, 1e-5, residual=residual)

    def _encode_sk(self, x: torch.Tensor, cu: torch.Tensor, T: int) -> torch.Tensor:
        """Encoder layers on the split-K tiled GEMM (no hipBLASLt): qkv (+ f32
        bias), flash attention, o (+ bias) added straight into the residual,
        LayerNorm, fc1 (+ bias, GELU), fc2 (+ bias) added into the residual."""
        cfg, w = self.cfg, self.w
        d, H, D = cfg.d_model, cfg.n_heads, cfg.head_dim
        residual = x.contiguous()
        for i, L in enumerate(w.enc):
            h = ops.layernorm(residual, L["ln1_w"], L["ln1_b"], 1e-5)
            qkv = ops.proj(h, L["wqkv"], bias=w.enc_qkv_bf[i])
            a = ops.attention(qkv, qkv[:, d:], qkv[:, 2 * d:], cu, n_heads=H, n_kv=H, head_dim=D,
                              causal=False, max_q=T, cu_k=cu)
            ops.proj(a, L["wo"], epi="resid", residual=residual, bias=w.enc_o_bf[i])
            h = ops.layernorm(residual, L["ln2_w"], L["ln2_b"], 1e-5)
            m = ops.proj(h, L["fc1"], bias=w.enc_fc1_bf[i], act="gelu")
            ops.proj(m, L["fc2"], epi="resid", residual=residual, bias=w.enc_fc2_bf[i])
        return ops.layernorm(residual, w.enc_ln_w, w.enc_ln_b, 1e-5)

    def cross_kv(self, enc: torch.Tensor) -> list[torch.Tensor]:
        """Per decoder layer [B*1500, 2d] cross-attention K|V (computed once)."""
        return [ops.linear(enc, L["xkv"], L["xkv_b"]) for L in self.w.dec]

    # ----------------------------------------------------------------- decoder
    def decode_step(self, tokens: torch.Tensor, positions: torch.Tensor, slots: torch.Tensor,
                    cu_q: torch.Tensor, ctx_lens: torch.Tensor, block_tables: torch.Tensor,
                    max_q: int, max_ctx: int, k_cache: torch.Tensor, v_cache: torch.Tensor,
                    xkv: list[torch.Tensor], enc_starts: torch.Tensor, enc_lens: torch.Tensor,
                    logit_idx: torch.Tensor, ws: ops.AttnWorkspace | None) -> torch.Tensor:
        """One decoder forward over a flat token batch; returns logits [B, V] of
        ``logit_idx`` rows. Self-attn K/V go to the paged cache (no RoPE)."""
        cfg, w = self.cfg, self.w
        d, H, D = cfg.d_model, cfg.n_heads, cfg.head_dim
        x = torch.nn.functional.embedding(tokens.long(), w.tok_embed)
        x = x + w.dec_pos.index_select(0, positions.long())
        residual = x
        h = ops.layernorm(x, w.dec[0]["ln1_w"], w.dec[0]["ln1_b"], 1e-5)
        delta = None
        enc_splits = (cfg.n_audio_ctx + 255) // 256
        self_splits = max(1, (max_ctx + 255) // 256)
        grouped = max_q <= 128
        for i, L in enumerate(w.dec):
            if i > 0:
                h = ops.layernorm(delta, L["ln1_w"], L["ln1_b"], 1e-5, residual=residual)
            qkv = ops.linear(h, L["wqkv"], L["bqkv"])
            ops.rope_kv_append(qkv, None, None, k_cache[i], v_cache[i], slots, H, H, D)
            a = ops.attention(qkv, k_cache[i], v_cache[i], cu_q, n_heads=H, n_kv=H, head_dim=D,
                              causal=True, max_q=max_q, ctx_lens=ctx_lens,
                              block_tables=block_tables, grouped=grouped, split_keys=256,
                              num_splits=self_splits if grouped else 1, workspace=ws,
                              max_k=max_ctx)
            o = ops.linear(a, L["wo"], L["bo"])
            h = ops.layernorm(o, L["lnx_w"], L["lnx_b"], 1e-5, residual=residual)
            q = ops.linear(h, L["xq"], L["xq_b"])
            kv = xkv[i]
            xa = ops.attention(q, kv, kv[:, d:], cu_q, n_heads=H, n_kv=H, head_dim=D, causal=False,
                               max_q=max_q, cu_k=enc_starts, ctx_lens=enc_lens,
                               grouped=grouped, split_keys=256,
                               num_splits=enc_splits if grouped else 1, workspace=ws)
            xo = ops.linear(xa, L["xo"], L["xo_b"])
            h = ops.layernorm(xo, L["ln2_w"], L["ln2_b"], 1e-5, residual=residual)
            m = ops.linear(h, L["fc1"], L["fc1_b"])
            ops.gelu_bias_(m)
            delta = ops.linear(m, L["fc2"], L["fc2_b"])
        sel_r = residual.index_select(0, logit_idx).contiguous()
        sel_d = delta.index_select(0, logit_idx).contiguous()
        hf = ops.layernorm(sel_d, w.dec_ln_w, w.dec_ln_b, 1e-5, residual=sel_r)
        return ops.linear(hf, w.tok_embed)


def decode_step_fast(model: "WhisperModel", tokens: torch.Tensor, positions: torch.Tensor,
                     slots: torch.Tensor, cu_q: torch.Tensor, ctx_lens: torch.Tensor,
                     block_tables: torch.Tensor, max_q: int, k_cache: torch.Tensor,
                     v_cache: torch.Tensor, xkv: list[torch.Tensor], enc_starts: torch.Tensor,
                     enc_lens: torch.Tensor, logit_idx: torch.Tensor, ws,
                     self_splits: int, split_keys: int = 128) -> torch.Tensor:
    """Decoder step on the weight-streaming path: every projection is the
    skinny split-K MFMA GEMM whose f32 slabs are reduced by the fused consumer
    that follows (bias + residual + LayerNorm, bias + KV append, bias + GELU);
    self- and cross-attention use the split-key decode kernel (cross-attention
    reads the encoder K/V rows in place). ``tokens`` has Mpad rows (padding
    rows carry slot -1); ``logit_idx`` has >= 16 rows. Graph-capturable: no
    host synchronisation, fixed ``self_splits``. Returns f32 logits
    [len(logit_idx), vocab_pad]."""
    cfg, w = model.cfg, model.w
    d, H, D = cfg.d_model, cfg.n_heads, cfg.head_dim
    enc_splits = (cfg.n_audio_ctx + split_keys - 1) // split_keys
    residual = ops.embed_pos(tokens, positions, w.tok_embed, w.dec_pos)
    h = ops.layernorm(residual, w.dec[0]["ln1_w"], w.dec[0]["ln1_b"], 1e-5)
    part = None
    for i, (L, P) in enumerate(zip(w.dec, w.dec_p)):
        if i > 0:
            h = ops.slab_layernorm(part, residual, L["ln1_w"], L["ln1_b"], 1e-5,
                                   bias=w.dec[i - 1]["fc2_b"])
        part = ops.skinny_gemm(h, P["wqkv"])
        q = ops.slab_rope_append(part, positions, None, k_cache[i], v_cache[i], slots, H, H, D,
                                 bias=L["bqkv"])
        a = ops.attention(q, k_cache[i], v_cache[i], cu_q, n_heads=H, n_kv=H, head_dim=D,
                          causal=True, max_q=max_q, ctx_lens=ctx_lens, block_tables=block_tables,
                          grouped=True, split_keys=split_keys, num_splits=self_splits,
                          workspace=ws)
        part = ops.skinny_gemm(a, P["wo"])
        h = ops.slab_layernorm(part, residual, L["lnx_w"], L["lnx_b"], 1e-5, bias=L["bo"])
        part = ops.skinny_gemm(h, P["xq"])
        q = ops.slab_bias_act(part, L["xq_b"])
        kv = xkv[i]
        a = ops.attention(q, kv, kv[:, d:], cu_q, n_heads=H, n_kv=H, head_dim=D, causal=False,
                          max_q=max_q, cu_k=enc_starts, ctx_lens=enc_lens, grouped=True,
                          split_keys=split_keys, num_splits=enc_splits, workspace=ws)
        part = ops.skinny_gemm(a, P["xo"])
        h = ops.slab_layernorm(part, residual, L["ln2_w"], L["ln2_b"], 1e-5, bias=L["xo_b"])
        part = ops.skinny_gemm(h, P["fc1"])
        m = ops.slab_bias_act(part, L["fc1_b"], "gelu")
        part = ops.skinny_gemm(m, P["fc2"])
    hf = ops.slab_layernorm(part, residual, w.dec_ln_w, w.dec_ln_b, 1e-5,
                            bias=w.dec[-1]["fc2_b"], row_idx=logit_idx, write_residual=False)
    return ops.skinny_gemm(hf, w.lm_head_p, 1, max_wgs=getattr(w, "max_wgs", ops.MAX_DECODE_WGS))[0]


def decode_step_fused(model: "WhisperModel", tokens: torch.Tensor, positions: torch.Tensor,
                      slots: torch.Tensor, cu_q: torch.Tensor, ctx_lens: torch.Tensor,
                      block_tables: torch.Tensor, max_q: int, k_cache: torch.Tensor,
                      v_cache: torch.Tensor, xkv: list[torch.Tensor], enc_starts: torch.Tensor,
                      enc_lens: torch.Tensor, logit_idx: torch.Tensor, ws, scratch,
                      self_splits: int, split_keys: int = 128,
                      cross_split_keys: int = 512) -> torch.Tensor:
    """Decoder step on the fused-epilogue GEMMs: 8 launches per layer.

    qkv   (LayerNorm ln1 prologue | bias + q / paged K,V append epilogue) ->
    self-attention -> o (bias + residual + row sum / sum-of-squares) ->
    xq    (LayerNorm lnx | bias) -> cross-attention over the encoder rows ->
    xo    (bias + residual + row stats) -> fc1 (LayerNorm ln2 | bias + GELU) ->
    fc2   (bias + residual + row stats).
    The LayerNorm statistics of a row come from the previous residual
    epilogue's per-tile partial sums, so no separate norm launch exists. Same
    contract as ``decode_step_fast``; Mpad (tokens rows) 16 or 32."""
    cfg, w = model.cfg, model.w
    d, H, D = cfg.d_model, cfg.n_heads, cfg.head_dim
    enc_splits = (cfg.n_audio_ctx + cross_split_keys - 1) // cross_split_keys
    Mpad = tokens.numel()
    if ops.FUSED_EMBED:
        residual = ops.embed_stats(tokens, w.tok_embed, scratch, positions=positions,
                                   pos_embed=w.dec_pos, sums=True)
    else:
        residual = ops.embed_pos(tokens, positions, w.tok_embed, w.dec_pos)
        scratch.seed_stats(residual)
    q = torch.empty(Mpad, H * D, dtype=torch.bfloat16, device=residual.device)
    for i, F in enumerate(w.dec_f):
        a = ops.skinny_fused(residual, F["qkv"], "rope", scratch, eps=1e-5, positions=positions,
                             q_out=q, k_cache=k_cache[i], v_cache=v_cache[i], slots=slots,
                             n_heads=H, n_kv=H, head_dim=D,
                             attn=dict(cu_q=cu_q, ctx_lens=ctx_lens, block_tables=block_tables,
                                       max_q=max_q, split_keys=split_keys,
                                       num_splits=self_splits, workspace=ws))
        ops.skinny_fused(a, F["o"], "resid", scratch, residual=residual, row_sums=True)
        kv = xkv[i]
        a = ops.skinny_fused(residual, F["xq"], "act", scratch, eps=1e-5, n_heads=H, n_kv=H,
                             head_dim=D,
                             attn=dict(cu_q=cu_q, ctx_lens=enc_lens, kv_start=enc_starts, k=kv,
                                       v=kv[:, d:], max_q=max_q, split_keys=cross_split_keys,
                                       num_splits=enc_splits, workspace=ws))
        ops.skinny_fused(a, F["xo"], "resid", scratch, residual=residual, row_sums=True)
        m = ops.skinny_fused(residual, F["fc1"], "act", scratch, act="gelu", eps=1e-5)
        ops.skinny_fused(m, F["fc2"], "resid", scratch, residual=residual, row_sums=True)
    if ops.FUSED_EMBED:
        hf = ops.layernorm(residual, w.dec_ln_w, w.dec_ln_b, 1e-5, row_idx=logit_idx)
    else:
        hf = ops.layernorm(residual.index_select(0, logit_idx), w.dec_ln_w, w.dec_ln_b, 1e-5)
    return ops.skinny_gemm(hf, w.lm_head_p, 1, max_wgs=getattr(w, "max_wgs", ops.MAX_DECODE_WGS))[0]


def pad_or_trim(audio: np.ndarray, n: int = 480000) -> np.ndarray:
    if len(audio) >= n:
        return audio[:n]
    return np.pad(audio, (0, n - len(audio)))
