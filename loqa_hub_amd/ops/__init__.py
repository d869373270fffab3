"""Hot ops of the voice hub.

Every op has two implementations:

* the **HIP kernel** (``csrc/kernels``, gfx950 MFMA/LDS) used whenever the inputs
  live on the GPU - a missing native library is a hard error there, never a
  silent fallback;
* a plain-PyTorch fp32 **reference** (``loqa_hub_amd.ops.reference``) used for
  CPU inputs (the CPU test tier, the config-1 plumbing path) and as the
  numerics oracle in ``tests/test_kernels_gpu.py``.

Plain GEMMs go to hipBLASLt through ``torch.nn.functional.linear``; every fused
elementwise/normalisation/attention/audio op around them is ours.
"""
from __future__ import annotations

import copy
import ctypes
import math
import os

import torch

from . import reference as ref
from . import _lib
from ._lib import FusedParams, check, kernels, ptr, stream_ptr


def _gpu(t: torch.Tensor) -> bool:
    return t.is_cuda


def _bf16_contig(t: torch.Tensor, name: str) -> None:
    if t.dtype != torch.bfloat16:
        raise TypeError(f"{name} must be bfloat16, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")


# --------------------------------------------------------------------- norms
def _norm_rows(x: torch.Tensor, residual, row_idx) -> tuple[int, int]:
    d = x.shape[-1]
    if row_idx is not None:
        # gathered rows: y[i] = norm(x[row_idx[i]]); no residual update then
        assert residual is None and x.dim() == 2
        assert row_idx.dtype == torch.int64 and row_idx.is_contiguous()
        return row_idx.numel(), d
    return x.numel() // d, d


def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float,
            residual: torch.Tensor | None = None,
            row_idx: torch.Tensor | None = None) -> torch.Tensor:
    """y = rmsnorm(x [+ residual]) * w; if residual is given it is updated in place
    to x + residual (the fused pre-norm residual stream). ``row_idx`` (int64)
    normalises only rows x[row_idx] (the decode step's logit rows) in the same
    launch."""
    if not _gpu(x):
        if row_idx is not None:
            x = x.index_select(0, row_idx.long())
        return ref.rmsnorm(x, w, eps, residual)
    rows, d = _norm_rows(x, residual, row_idx)
    _bf16_contig(x, "x"); _bf16_contig(w, "w")
    if residual is not None:
        _bf16_contig(residual, "residual")
        assert residual.shape == x.shape
    assert w.numel() == d
    y = torch.empty((rows, d) if row_idx is not None else x.shape, dtype=x.dtype, device=x.device)
    check(kernels().loqa_rmsnorm(ptr(x), ptr(residual), ptr(w), ptr(y), rows, d, eps,
                                 ptr(row_idx), stream_ptr(x)), "rmsnorm")
    return y


def layernorm(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, eps: float,
              residual: torch.Tensor | None = None,
              row_idx: torch.Tensor | None = None) -> torch.Tensor:
    """y = layernorm(x [+ residual]) * w + b; ``residual`` / ``row_idx`` as in
    :func:`rmsnorm`."""
    if not _gpu(x):
        if row_idx is not None:
            x = x.index_select(0, row_idx.long())
        return ref.layernorm(x, w, b, eps, residual)
    rows, d = _norm_rows(x, residual, row_idx)
    _bf16_contig(x, "x"); _bf16_contig(w, "w"); _bf16_contig(b, "b")
    if residual is not None:
        _bf16_contig(residual, "residual")
        assert residual.shape == x.shape
    y = torch.empty((rows, d) if row_idx is not None else x.shape, dtype=x.dtype, device=x.device)
    check(kernels().loqa_layernorm(ptr(x), ptr(residual), ptr(w), ptr(b), ptr(y), rows, d, eps,
                                   ptr(row_idx), stream_ptr(x)), "layernorm")
    return y


# --------------------------------------------------------------- elementwise
def silu_mul(x: torch.Tensor) -> torch.Tensor:
    """x: [..., 2F] = [gate | up] -> silu(gate) * up: [..., F]"""
    if not _gpu(x):
        return ref.silu_mul(x)
    _bf16_contig(x, "x")
    F = x.shape[-1] // 2
    rows = x.numel() // (2 * F)
    out = torch.empty(*x.shape[:-1], F, dtype=x.dtype, device=x.device)
    check(kernels().loqa_silu_mul(ptr(x), ptr(out), rows, F, stream_ptr(x)), "silu_mul")
    return out


def gelu_bias_(x: torch.Tensor, bias: torch.Tensor | None = None,
               pos: torch.Tensor | None = None) -> torch.Tensor:
    """In place: x = gelu(x + bias) [+ pos[row % pos.shape[0]]]."""
    if not _gpu(x):
        return ref.gelu_bias_(x, bias, pos)
    _bf16_contig(x, "x")
    F = x.shape[-1]
    rows = x.numel() // F
    if bias is not None:
        _bf16_contig(bias, "bias"); assert bias.numel() == F
    period = 0
    if pos is not None:
        _bf16_contig(pos, "pos"); assert pos.shape[-1] == F
        period = pos.shape[0]
    check(kernels().loqa_gelu_bias(ptr(x), ptr(bias), ptr(pos), rows, F, period, stream_ptr(x)),
          "gelu_bias")
    return x


def rope_kv_append(qkv: torch.Tensor, positions: torch.Tensor | None, cos_sin: torch.Tensor | None,
                   k_cache: torch.Tensor, v_cache: torch.Tensor, slots: torch.Tensor,
                   n_heads: int, n_kv: int, head_dim: int) -> None:
    """Rotate q (in place in ``qkv``) and k, and append k/v to the paged cache.

    qkv: [T, >= (H + 2 Hkv) * D] bf16; positions/slots: [T] int32;
    cos_sin: [max_pos, D/2, 2] f32 or None (no rotation);
    caches: [n_blocks, Hkv, BLK, D] bf16.
    """
    if not _gpu(qkv):
        return ref.rope_kv_append(qkv, positions, cos_sin, k_cache, v_cache, slots, n_heads, n_kv,
                                  head_dim)
    T = qkv.shape[0]
    if T == 0:
        return None
    assert qkv.dtype == torch.bfloat16 and qkv.stride(-1) == 1
    assert qkv.shape[1] >= (n_heads + 2 * n_kv) * head_dim
    assert slots.dtype == torch.int32 and slots.numel() == T and slots.is_contiguous()
    if cos_sin is not None:
        assert positions is not None and positions.dtype == torch.int32 and positions.numel() == T
        assert cos_sin.dtype == torch.float32 and cos_sin.shape[-2] == head_dim // 2
    assert k_cache.shape[1] == n_kv and k_cache.shape[3] == head_dim and k_cache.is_contiguous()
    blk = k_cache.shape[2]
    check(kernels().loqa_rope_kv_append(ptr(qkv), qkv.stride(0), ptr(positions), ptr(cos_sin),
                                        ptr(k_cache), ptr(v_cache), ptr(slots), T, n_heads, n_kv,
                                        head_dim, blk, stream_ptr(qkv)), "rope_kv_append")
    return None


# ----------------------------------------------------------------- attention
class AttnWorkspace:
    """Split-K partial buffers for grouped decode attention (allocated once per
    engine so the decode step stays graph-capturable)."""

    def __init__(self, device, max_tokens: int, n_heads: int, head_dim: int, max_splits: int):
        self.max_tokens, self.max_splits = max_tokens, max_splits
        self.part_o = torch.empty(max_splits * max_tokens * n_heads * head_dim, dtype=torch.float32,
                                  device=device)
        self.part_ml = torch.empty(max_splits * max_tokens * n_heads * 2, dtype=torch.float32,
                                   device=device)
        # split-arrival tickets of the decode kernel's in-launch combine, one per
        # (sequence, kv head); the last arriving split resets its counter
        self.counters = torch.zeros(max_tokens * n_heads, dtype=torch.int32, device=device)


# decode attention (attn_decode.hip): splits of at least this many keys run on
# 8-wave workgroups (0: always 4 waves)
ATTN8_MIN_KEYS = int(os.environ.get("LOQA_ATTN8_MIN_KEYS", "0"))
# splits of at least this many keys (and more than one tile per wave) prefetch
# a wave's next K / V tile (4 waves: one per SIMD; 0: never)
ATTN_PF_MIN_KEYS = int(os.environ.get("LOQA_ATTN_PF_MIN_KEYS", "0"))


def attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, cu_q: torch.Tensor, *,
              n_heads: int, n_kv: int, head_dim: int, causal: bool, max_q: int,
              cu_k: torch.Tensor | None = None, ctx_lens: torch.Tensor | None = None,
              block_tables: torch.Tensor | None = None, scale: float | None = None,
              grouped: bool = False, split_keys: int = 256, num_splits: int = 1,
              workspace: AttnWorkspace | None = None, out: torch.Tensor | None = None,
              max_k: int | None = None) -> torch.Tensor:
    """Varlen flash attention.

    q: [Tq, >=H*D] (row stride may exceed H*D, e.g. a view into the fused QKV
    output). K/V: contiguous [Tk, >=Hkv*D] with ``cu_k``, or paged caches
    [n_blocks, Hkv, BLK, D] with ``ctx_lens`` + ``block_tables``.
    Query i of sequence b sits at absolute position ctx_len_b - q_len_b + i.
    Returns [Tq, H*D] bf16.
    """
    scale = scale if scale is not None else 1.0 / math.sqrt(head_dim)
    if not _gpu(q):
        return ref.attention(q, k, v, cu_q, n_heads=n_heads, n_kv=n_kv, head_dim=head_dim,
                             causal=causal, cu_k=cu_k, ctx_lens=ctx_lens,
                             block_tables=block_tables, scale=scale, out=out)
    Tq = q.shape[0]
    B = cu_q.numel() - 1
    if out is None:
        out = torch.empty(Tq, n_heads * head_dim, dtype=torch.bfloat16, device=q.device)
    if Tq == 0 or B == 0:
        return out
    assert q.dtype == torch.bfloat16 and q.stride(-1) == 1 and q.shape[1] >= n_heads * head_dim
    assert cu_q.dtype == torch.int32 and cu_q.is_contiguous()
    assert out.stride(-1) == 1 and out.shape[0] == Tq
    paged = block_tables is not None
    if paged:
        assert k.dim() == 4 and k.shape[1] == n_kv and k.shape[3] == head_dim and k.is_contiguous()
        assert v.shape == k.shape and v.is_contiguous()
        assert ctx_lens is not None and ctx_lens.dtype == torch.int32 and ctx_lens.numel() == B
        assert block_tables.dtype == torch.int32 and block_tables.is_contiguous()
        assert block_tables.shape[0] == B
        blk, max_blocks, kv_stride = k.shape[2], block_tables.shape[1], 0
        if max_k is not None:
            assert max_k <= max_blocks * blk, "context exceeds block table"
    else:
        assert cu_k is not None and cu_k.dtype == torch.int32
        if ctx_lens is None:
            assert cu_k.numel() == B + 1
        else:  # explicit per-sequence starts (cu_k) and lengths (ctx_lens)
            assert cu_k.numel() >= B and ctx_lens.dtype == torch.int32 and ctx_lens.numel() == B
        assert k.stride(-1) == 1 and v.stride(-1) == 1 and k.stride(0) == v.stride(0)
        blk, max_blocks, kv_stride = 0, 0, k.stride(0)
    part_o = part_ml = None
    if grouped and (n_heads // n_kv) * max_q <= 32 and split_keys % 32 == 0 and \
            (paged or ctx_lens is not None):
        # split-key decode kernel (attn_decode.hip): paged cache, or contiguous
        # rows at per-sequence starts cu_k[b] with lengths ctx_lens[b]
        assert workspace is not None and workspace.max_splits >= num_splits
        assert workspace.max_tokens >= Tq and B * n_kv <= workspace.counters.numel()
        assert not paged or (blk >= 16 and blk & (blk - 1) == 0)
        kv_stride = 0 if paged else k.stride(0)
        # a split of >= ATTN8_MIN_KEYS keys runs on 8 waves (256 keys per
        # pass); with more than 256 keys a wave also prefetches its next tile
        waves = 8 if (ATTN8_MIN_KEYS and split_keys >= ATTN8_MIN_KEYS) else 4
        pf = int(split_keys > 32 * waves and ATTN_PF_MIN_KEYS and split_keys >= ATTN_PF_MIN_KEYS)
        check(kernels().loqa_attn_decode(
            ptr(q), q.stride(0), ptr(k), ptr(v), kv_stride, None if paged else ptr(cu_k),
            ptr(out), out.stride(0), ptr(cu_q), ptr(ctx_lens),
            ptr(block_tables) if paged else None, max_blocks, blk, B, max_q, n_heads, n_kv,
            head_dim, scale, int(causal), split_keys, num_splits, ptr(workspace.part_o),
            ptr(workspace.part_ml), Tq, ptr(workspace.counters), waves, pf, stream_ptr(q)),
            "attn_decode")
        return out
    if grouped:
        G = n_heads // n_kv
        assert max_q * G <= 128, "grouped attention handles at most 128/G query tokens"
        if num_splits > 1:
            assert workspace is not None and workspace.max_splits >= num_splits
            assert workspace.max_tokens >= Tq
            part_o, part_ml = workspace.part_o, workspace.part_ml
    check(kernels().loqa_attention(
        ptr(q), q.stride(0), ptr(k), ptr(v), kv_stride, ptr(out), out.stride(0), ptr(cu_q),
        ptr(cu_k), ptr(ctx_lens), ptr(block_tables), max_blocks, blk, B, max_q, n_heads, n_kv,
        head_dim, scale, int(causal), int(grouped), split_keys, num_splits, ptr(part_o),
        ptr(part_ml), Tq, stream_ptr(q)), "attention")
    return out


# ----------------------------------------------------------------- sampling
def masked_argmax(logits: torch.Tensor, mask: torch.Tensor | None = None,
                  mask_rows: torch.Tensor | None = None) -> torch.Tensor:
    """argmax over tokens allowed by a packed uint32 bitmask (bit v%32 of word
    v//32). ``mask_rows`` optionally maps each logits row to a mask-table row.
    Returns int32 [B] (-1 if nothing is allowed)."""
    if not _gpu(logits):
        return ref.masked_argmax(logits, mask, mask_rows)
    assert logits.dim() == 2 and logits.stride(-1) == 1
    B, V = logits.shape
    W = 0
    if mask is not None:
        assert mask.dtype == torch.int32 and mask.is_contiguous()
        W = mask.shape[-1]
        assert W * 32 >= V
        if mask_rows is not None:
            assert mask_rows.dtype == torch.int32 and mask_rows.numel() == B
        else:
            assert mask.shape[0] >= B
    is_bf16 = logits.dtype == torch.bfloat16
    assert is_bf16 or logits.dtype == torch.float32
    out = torch.empty(B, dtype=torch.int32, device=logits.device)
    ws = torch.empty(B, dtype=torch.int64, device=logits.device)
    check(kernels().loqa_masked_argmax(ptr(logits), int(is_bf16), logits.stride(0), B, V,
                                       ptr(mask), ptr(mask_rows), W, ptr(out), ptr(ws),
                                       stream_ptr(logits)), "masked_argmax")
    return out


# -------------------------------------------------------------------- audio
def pcm16_to_f32_sumsq(pcm: torch.Tensor, offsets: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """pcm: int16 [N] (concatenated segments), offsets: int64 [S+1].
    Returns (f32 samples [N] = x/32767, per-segment sum of squares [S])."""
    if not _gpu(pcm):
        return ref.pcm16_to_f32_sumsq(pcm, offsets)
    assert pcm.dtype == torch.int16 and pcm.is_contiguous()
    assert offsets.dtype == torch.int64 and offsets.is_contiguous()
    S = offsets.numel() - 1
    out = torch.empty(pcm.numel(), dtype=torch.float32, device=pcm.device)
    sumsq = torch.empty(max(S, 1), dtype=torch.float32, device=pcm.device)
    seg = offsets.cpu()
    max_len = int((seg[1:] - seg[:-1]).max()) if S > 0 else 0
    assert int(seg[-1]) <= pcm.numel()
    check(kernels().loqa_pcm16_f32_sumsq(ptr(pcm), ptr(out), ptr(offsets), ptr(sumsq), S, max_len,
                                         stream_ptr(pcm)), "pcm16_f32_sumsq")
    return out, sumsq[:S]


def pcm16_to_f32_padded(pcm: torch.Tensor, offsets: torch.Tensor, ld: int,
                        offsets_host: "np.ndarray | None" = None) -> tuple[torch.Tensor, torch.Tensor]:
    """pcm int16 [N] (S concatenated segments, offsets int64 [S+1]) -> f32
    [S, ld] (x / 32767, zero-padded / truncated to ``ld`` samples) and the
    per-segment sum of squares [S] of the kept samples."""
    S = offsets.numel() - 1
    if not _gpu(pcm):
        out = torch.zeros(S, ld, dtype=torch.float32)
        seg = offsets.cpu()
        for i in range(S):
            n = min(int(seg[i + 1] - seg[i]), ld)
            out[i, :n] = pcm[int(seg[i]):int(seg[i]) + n].float() / 32767.0
        return out, out.square().sum(1)
    assert pcm.dtype == torch.int16 and pcm.is_contiguous()
    assert offsets.dtype == torch.int64 and offsets.is_contiguous() and offsets.is_cuda
    out = torch.empty(S, ld, dtype=torch.float32, device=pcm.device)
    sumsq = torch.empty(max(S, 1), dtype=torch.float32, device=pcm.device)
    if offsets_host is not None:
        assert int(offsets_host[-1]) <= pcm.numel()
    check(kernels().loqa_pcm16_f32_pad(ptr(pcm), ptr(out), ptr(offsets), ptr(sumsq), S, ld,
                                       stream_ptr(pcm)), "pcm16_f32_pad")
    return out, sumsq[:S]


def log_mel(audio: torch.Tensor, consts: "ref.MelConstants") -> torch.Tensor:
    """audio [B, n_samples] f32 (padded to 30 s) -> whisper log-mel [B, n_mels, frames] bf16."""
    if not _gpu(audio):
        return ref.log_mel(audio, consts).to(torch.bfloat16)
    assert audio.dtype == torch.float32 and audio.is_contiguous() and audio.dim() == 2
    B, n = audio.shape
    frames = n // 160
    c = consts.to(audio.device)
    work = torch.empty(B, c.n_mels, frames, dtype=torch.float32, device=audio.device)
    gmax = torch.empty(B, dtype=torch.float32, device=audio.device)
    out = torch.empty(B, c.n_mels, frames, dtype=torch.bfloat16, device=audio.device)
    check(kernels().loqa_log_mel(ptr(audio), B, n, ptr(c.window), ptr(c.cos_basis),
                                 ptr(c.sin_basis), ptr(c.filters), c.n_mels, ptr(work), ptr(gmax),
                                 ptr(out), frames, stream_ptr(audio)), "log_mel")
    return out


def im2col_k3(x: torch.Tensor, strides: tuple[int, int, int], B: int, C: int, L: int,
              stride: int) -> torch.Tensor:
    """Unfold a k=3/pad=1 conv1d input. x element (b,c,t) at
    b*strides[0] + c*strides[1] + t*strides[2]. Returns [B*Lout, 3C] bf16."""
    Lout = (L - 1) // stride + 1
    if not _gpu(x):
        return ref.im2col_k3(x, strides, B, C, L, stride)
    assert x.dtype == torch.bfloat16
    cols = torch.empty(B * Lout, 3 * C, dtype=torch.bfloat16, device=x.device)
    check(kernels().loqa_im2col_k3(ptr(x), strides[0], strides[1], strides[2], B, C, L, stride,
                                   ptr(cols), stream_ptr(x)), "im2col_k3")
    return cols


def tensor_seed(seed: int, *key) -> int:
    """uint32 stream id of one weight tensor of a seeded random init (stable
    across processes and Python versions: no ``hash()``)."""
    h = (seed * 0x9E3779B1 + 0x7F4A7C15) & 0xFFFFFFFF
    for k in key:
        for ch in str(k).encode():
            h = ((h ^ ch) * 0x01000193) & 0xFFFFFFFF
        h = ((h ^ 0xFF) * 0x01000193) & 0xFFFFFFFF
    return h


def init_normal(rows: int, cols: int, *, seed: int, key: tuple, std: float = 0.02,
                ld: int | None = None, row0: int = 0, col0: int = 0, device="cpu") -> torch.Tensor:
    """Seeded random-init block [rows, cols] bf16 of a conceptual [*, ld] tensor
    at (row0, col0): zero mean, standard deviation ``std`` (Irwin-Hall(4), a
    near-normal with bounded tails). A shard generated on its own holds
    exactly the values of the unsharded tensor, on the GPU and the CPU alike."""
    ld = cols if ld is None else ld
    s = tensor_seed(seed, *key)
    scale = float(torch.tensor(std * math.sqrt(3.0), dtype=torch.float32))
    dev = torch.device(device)
    if dev.type != "cuda":
        return ref.init_uniform4(rows, cols, ld, row0, col0, s, scale).to(dev)
    out = torch.empty(rows, cols, dtype=torch.bfloat16, device=dev)
    check(kernels().loqa_init_uniform4(ptr(out), rows, cols, ld, row0, col0, s, scale,
                                       stream_ptr(out)), "init_uniform4")
    return out


def linear(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None = None) -> torch.Tensor:
    """Plain GEMM: hipBLASLt via torch on the GPU."""
    return torch.nn.functional.linear(x, w, b)


# ------------------------------------------------- decode GEMM + slab consumers
MPADS = (16, 32, 64, 128)


def mpad_for(m: int) -> int:
    for p in MPADS:
        if m <= p:
            return p
    raise ValueError(f"skinny GEMM supports at most {MPADS[-1]} rows, got {m}")


_SPLITS: dict[tuple[int, int, int], int] = {}
# K must be a multiple of S * 128 (4 waves x 32-wide k-steps); 5 and 10 cover
# Whisper's K = 1280 (= 10 * 128)
SPLIT_CANDIDATES = (1, 2, 4, 5, 8, 10)


def tune_skinny_splits(wp: torch.Tensor, mpads=MPADS, reps: int = 8) -> dict:
    """Time the skinny GEMM for every split-K option on the real weight and
    cache the fastest per (N, K, Mpad). Per-CU bandwidth (~24 GB/s per CU) makes
    grid balance across the 256 CUs the dominant effect, and it depends on the
    shape, so it is measured rather than modelled. Run before graph capture."""
    N, K = wp.shape[0] * 16, wp.shape[1] * 32
    if not _gpu(wp) or NO_TUNE:
        return {}
    out = {}
    for Mpad in mpads:
        key = (N, K, Mpad)
        if key in _SPLITS:
            out[key] = _SPLITS[key]
            continue
        x = torch.randn(Mpad, K, device=wp.device, dtype=torch.bfloat16)
        best, best_t = 1, float("inf")
        for s in SPLIT_CANDIDATES:
            if K % (s * 128):
                continue
            t = graph_time(lambda: skinny_gemm(x, wp, s), reps)
            if t < best_t * 0.98:
                best, best_t = s, t
        _SPLITS[key] = best
        out[key] = best
    return out


_FSPLITS: dict = {}
MAX_DECODE_WGS = int(os.environ.get("LOQA_MAX_DECODE_WGS", "256"))
# LOQA_NO_TUNE=1: skip every split-K / layout measurement and use the
# heuristic defaults (processes sharing one GPU - e.g. a TP rehearsal on a
# 1-GPU box - cannot time anything meaningful, and the timing dominates start-up)
NO_TUNE = os.environ.get("LOQA_NO_TUNE", "0") == "1"
# fused-GEMM decode steps: embedding + layer-0 row statistics in one launch and
# the final norm gathering its logit rows itself (False: the unfused torch ops)
FUSED_EMBED = True
_CAP = [MAX_DECODE_WGS]   # active co-scheduling cap while tuning (see decode_cap)


class decode_cap:
    """Context: tune decode GEMMs for a grid of at most ``n`` workgroups (an
    engine confined to n CUs by a CU mask gets n; default MAX_DECODE_WGS)."""

    def __init__(self, n: int | None):
        self.n = n or MAX_DECODE_WGS

    def __enter__(self):
        self.prev = _CAP[0]
        _CAP[0] = self.n
        return self

    def __exit__(self, *exc):
        _CAP[0] = self.prev


def _fsplit_override(key: tuple) -> tuple[int, int, int] | None:
    """``LOQA_FSPLIT_OVERRIDE="silu:28672x4096:M16=2,2,1;..."`` pins the
    (split-K, rt, wr) of a fused GEMM shape (experiments / deployment pins)."""
    spec = os.environ.get("LOQA_FSPLIT_OVERRIDE", "")
    name = f"{key[0]}:{key[1]}x{key[2]}:M{key[3]}"
    for item in spec.split(";"):
        if "=" in item:
            k, v = item.split("=", 1)
            if k.strip() == name:
                return tuple(int(t) for t in v.split(","))
    return None


class contended_tuning:
    """Context: while tuning, keep a Llama-3-8B-like gate|up weight stream
    (rows-per-wave fused GEMM over ~700 MB of cold weights) running on a
    background stream. The Whisper decoder always runs beside the LLM decode;
    its kernels' best split-K / tile shape under that load differs from the
    isolated optimum (split-K hand-offs cost extra memory round trips that
    queue behind the co-resident weight stream)."""

    def __init__(self, device, enabled: bool = True):
        self.device, self.enabled = torch.device(device), enabled

    def __enter__(self):
        if not (self.enabled and self.device.type == "cuda"):
            return self
        import threading
        dev = self.device
        bf = dict(dtype=torch.bfloat16, device=dev)
        self._ws = [shuffle_weight(torch.randn(28672, 4096, **bf) * 0.02) for _ in range(3)]
        self._x = torch.randn(16, 4096, **bf)
        self._scr = FusedScratch(dev)
        self._scr.rowsq[: 128 * 16].fill_(32.0)
        self._stop = threading.Event()
        self._stream = torch.cuda.Stream(dev)
        ready = threading.Event()

        # the background work is one captured graph, replayed and paced by
        # event polling: no synchronising HIP call while the tuner captures
        with torch.cuda.stream(self._stream):
            for i in range(3):
                skinny_fused(self._x, self._ws[i], "silu", self._scr, splits=1, rt=2, wr=4, norm=True,
                             rowsq_tiles=128)
        self._stream.synchronize()
        self._g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self._g, stream=self._stream):
            for i in range(12):
                skinny_fused(self._x, self._ws[i % 3], "silu", self._scr, splits=1, rt=2, wr=4,
                             norm=True, rowsq_tiles=128)

        def loop():
            import time as _time
            torch.cuda.set_device(dev)
            with torch.cuda.stream(self._stream):
                while not self._stop.is_set():
                    self._g.replay()
                    ev = torch.cuda.Event()
                    ev.record(self._stream)
                    while not ev.query():
                        _time.sleep(0.0002)
                    ready.set()
        self._th = threading.Thread(target=loop, daemon=True)
        self._th.start()
        ready.wait(30)
        return self

    def __exit__(self, *exc):
        if getattr(self, "_th", None) is not None:
            self._stop.set()
            self._th.join()
            torch.cuda.synchronize(self.device)
            del self._g, self._ws, self._x, self._scr
            self._th = None


def tune_fused_splits(key: tuple, run, K: int, reps: int = 8, rts=(2,), ncopies: int = 1,
                      wr4: bool = False, fewest: bool = True, xl: str = "no",
                      splits: list | None = None) -> tuple:
    """(split-K, tile rows / 16, waves along rows) for a fused-epilogue GEMM,
    measured: ``run(s, rt, wr, i)`` launches it on weight copy ``i`` (the graph
    cycles through ``ncopies`` copies so every call streams COLD weights, as a
    decode step that reads the whole model does; a warm replay of one copy is
    partly served by the 256 MB Infinity Cache and ranks the options wrongly).
    The in-launch reduce adds a store-drain + ticket round trip to every
    workgroup's tail, so the best split is lower than the plain GEMM's; 16-row
    tiles (rt=1, residual / act epilogues only) double the workgroups without
    any reduction; ``wr4`` adds the 4-waves-along-rows layout (S = 1 only). ``xl``: "no",
    "also" (add the x-through-LDS layouts, any split) or "only" (Mpad 128).
    Returns (split-K, rt, wr) or (split-K, rt, 4, 1) for an XL layout.
    ``key`` = (mode, N, K, Mpad)."""
    if key in _FSPLITS:
        return _FSPLITS[key]
    ov = _fsplit_override(key)
    if ov is not None:
        _FSPLITS[key] = ov
        return ov
    N = key[1]
    cands = [] if xl == "only" else \
        [(s, rt, 1) for rt in rts for s in (splits or SPLIT_CANDIDATES) if K % (s * 128) == 0]
    if wr4 and xl != "only":
        cands += [(1, rt, 4) for rt in rts if N % (64 * rt) == 0]
    if xl != "no":
        cands += [(s, rt, 4, 1) for rt in (1, 2) for s in SPLIT_CANDIDATES
                  if K % (s * 128) == 0 and N % (64 * rt) == 0]
    # co-scheduling cap: the STT and LLM decoders run concurrently on their own
    # streams; a grid that fills every CU slot makes the other stream's small
    # latency-bound kernels wait for it to drain (measured: a 768-workgroup
    # qkv GEMM, fastest in isolation, slowed the concurrent Whisper decoder 5x
    # and the whole pipeline 1.8x). Keep at most one workgroup per CU.
    units = {c: (N // (16 * c[1] * c[2])) * c[0] for c in cands}
    capped = [c for c in cands if units[c] <= _CAP[0]]
    if not capped and fewest:
        # a GEMM too large for any layout under the cap (Llama-3-70B gate|up:
        # >= 448 workgroups) takes the fewest-workgroup layouts (measured cold,
        # 70B gate|up: 448 WGs 154 us vs 3584 WGs 169 us)
        least = min(units.values())
        capped = [c for c in cands if units[c] <= max(_CAP[0], 2 * least)]
    elif not capped:
        # Llama-3-8B gate|up at Mpad 64 (jump-forward decode steps beside the
        # Whisper decoder): the short-lived 16-row tiles. Measured in the
        # pipeline: 18.9 utt/s, vs 17.2 for 896 longer 32-row workgroups
        # (fastest alone) and 11.0 for 224 4-wave 32-row workgroups.
        capped = cands[:1]
    cands = capped
    best, best_t = cands[0] if xl == "only" else (1, rts[-1], 1), float("inf")
    n = max(1, ncopies)
    for c in cands:
        it = iter(range(1 << 30))
        t = graph_time(lambda: run(*c[:3], next(it) % n, *c[3:]), max(reps, 2 * n))
        if t < best_t * 0.98:
            best, best_t = c, t
    _FSPLITS[key] = best
    return best


_TUNE_STREAM: dict = {}


def _tune_stream() -> "torch.cuda.Stream":
    """One side stream per device for every tuning capture. ``torch.cuda.Stream()``
    and ``torch.cuda.graph()`` without a stream take the NEXT stream of
    PyTorch's round-robin pool, and pool streams land on the process's few HIP
    hardware queues in creation order: a tuner that drew one pool stream per
    candidate left the decoder streams created after it on queues that
    depended on how many layouts were timed (see docs/PERF.md, the cliff)."""
    d = torch.cuda.current_device()
    if d not in _TUNE_STREAM:
        _TUNE_STREAM[d] = torch.cuda.Stream()
    return _TUNE_STREAM[d]


def graph_time(fn, reps: int = 8, trials: int = 3) -> float:
    """Device time (ms) of ``reps`` back-to-back calls of ``fn`` replayed from
    a captured HIP graph (no host launch overhead in the measurement: a few-µs
    kernel is otherwise hidden behind its own launch cost); min over trials."""
    # A new pool stream per call, on purpose: the stream-pool cursor this
    # leaves behind decides which hardware queues the decoder streams created
    # later land on, and the measured-best placement (18.7-19.2 utt/s) is the
    # one this produces. A fixed tuning stream (``_tune_stream``) measured
    # 17.3 (docs/PERF.md, "the 1.8x cliff").
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(trials):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        b.synchronize()
        best = min(best, a.elapsed_time(b))
    del g
    return best


def choose_splits(N: int, K: int, Mpad: int, target_wgs: int = 512) -> int:
    """Split-K factor: the tuned value if available, else enough splits for
    >= ~2 workgroups per CU (256 CUs)."""
    tuned = _SPLITS.get((N, K, Mpad))
    if tuned is not None:
        return tuned
    rt = 2 if Mpad <= 32 else 4
    tiles = max(1, N // (16 * rt))
    best = 1
    for s in SPLIT_CANDIDATES:
        if K % (s * 128) != 0:
            continue
        best = s
        if tiles * s >= target_wgs:
            break
    return best


def decode_attn_splits(max_ctx: int, units: int, split_keys: int = 128,
                       max_wgs: int | None = None) -> tuple[int, int]:
    """(num_splits, split_keys) of the split-key decode attention for a
    context bound and ``units`` = sequences x kv heads workgroup rows: splits of
    ``split_keys`` keys, but at most ``max_wgs`` workgroups in all (the
    co-scheduling cap of ``tune_fused_splits``) - longer splits then loop."""
    max_wgs = MAX_DECODE_WGS if max_wgs is None else max_wgs
    ns = max(1, -(-max_ctx // split_keys))
    cap = max(1, max_wgs // max(1, units))
    if ns > cap:
        ns = cap
        split_keys = -(-(-(-max_ctx // ns)) // 32) * 32
    return ns, split_keys


def shuffle_weight(w: torch.Tensor) -> torch.Tensor:
    """[N, K] bf16 -> MFMA-fragment-ordered [N/16, K/32, 64, 8] (skinny GEMM layout)."""
    N, K = w.shape
    assert N % 16 == 0 and K % 32 == 0
    if not _gpu(w):
        return ref.shuffle_weight(w)
    _bf16_contig(w, "w")
    out = torch.empty(N // 16, K // 32, 64, 8, dtype=torch.bfloat16, device=w.device)
    check(kernels().loqa_shuffle_weight(ptr(w), ptr(out), N, K, stream_ptr(w)), "shuffle_weight")
    return out


def skinny_gemm(x: torch.Tensor, wp: torch.Tensor, splits: int | None = None,
                max_wgs: int = 0) -> torch.Tensor:
    """x [Mpad, K] bf16 (Mpad in 16/32/64/128, padded rows finite) @ W^T with W
    given pre-shuffled (``shuffle_weight``) -> split-K partial slabs
    [S, Mpad, N] f32 (sum over S = x @ W^T)."""
    Mpad, K = x.shape
    N = wp.shape[0] * 16
    assert wp.shape[1] * 32 == K, "weight/activation K mismatch"
    S = splits or choose_splits(N, K, Mpad)
    if not _gpu(x):
        return ref.skinny_gemm(x, wp, S)
    assert Mpad in MPADS and x.dtype == torch.bfloat16 and x.stride(1) == 1
    _bf16_contig(wp, "wp")
    part = torch.empty(S, Mpad, N, dtype=torch.float32, device=x.device)
    check(kernels().loqa_skinny_gemm(ptr(x), x.stride(0), ptr(wp), ptr(part), Mpad, N, K, S,
                                     max_wgs, stream_ptr(x)), "skinny_gemm")
    return part


def slab_rmsnorm(part: torch.Tensor, residual: torch.Tensor, w: torch.Tensor, eps: float,
                 row_idx: torch.Tensor | None = None, write_residual: bool = True) -> torch.Tensor:
    """residual[src] += sum_s part[s, src]; y[i] = rmsnorm(residual[src]) * w with
    src = row_idx[i] (or i). Returns y [rows, d] bf16."""
    S, Mpad, d = part.shape
    rows = row_idx.numel() if row_idx is not None else Mpad
    if not _gpu(part):
        return ref.slab_rmsnorm(part, residual, w, eps, row_idx, write_residual)
    assert part.dtype == torch.float32 and part.is_contiguous()
    _bf16_contig(residual, "residual")
    assert residual.shape[-1] == d and residual.shape[0] >= Mpad
    if row_idx is not None:
        assert row_idx.dtype == torch.int64 and row_idx.is_contiguous()
    y = torch.empty(rows, d, dtype=torch.bfloat16, device=part.device)
    check(kernels().loqa_slab_rmsnorm(ptr(part), S, Mpad, ptr(row_idx), rows, ptr(residual),
                                      int(write_residual), ptr(w), ptr(y), d, eps,
                                      stream_ptr(part)), "slab_rmsnorm")
    return y


def slab_rope_append(part: torch.Tensor, positions: torch.Tensor, cos_sin: torch.Tensor | None,
                     k_cache: torch.Tensor, v_cache: torch.Tensor, slots: torch.Tensor,
                     n_heads: int, n_kv: int, head_dim: int,
                     bias: torch.Tensor | None = None) -> torch.Tensor:
    """qkv slabs [S, Mpad, (H+2Hkv)D] (+ optional projection bias) -> rotated q
    [Mpad, H*D] bf16; k/v to cache (``cos_sin`` None = no rotary embedding)."""
    S, Mpad, N = part.shape
    assert N == (n_heads + 2 * n_kv) * head_dim
    if not _gpu(part):
        return ref.slab_rope_append(part, positions, cos_sin, k_cache, v_cache, slots, n_heads,
                                    n_kv, head_dim, bias)
    assert slots.dtype == torch.int32 and slots.numel() == Mpad
    assert positions.dtype == torch.int32 and positions.numel() == Mpad
    assert k_cache.is_contiguous() and k_cache.shape[1] == n_kv and k_cache.shape[3] == head_dim
    q = torch.empty(Mpad, n_heads * head_dim, dtype=torch.bfloat16, device=part.device)
    check(kernels().loqa_slab_rope_append(ptr(part), S, Mpad, Mpad, ptr(positions), ptr(cos_sin),
                                          ptr(q), ptr(k_cache), ptr(v_cache), ptr(slots), n_heads,
                                          n_kv, head_dim, k_cache.shape[2], ptr(bias),
                                          stream_ptr(part)),
          "slab_rope_append")
    return q


def slab_layernorm(part: torch.Tensor, residual: torch.Tensor, w: torch.Tensor, b: torch.Tensor,
                   eps: float, bias: torch.Tensor | None = None,
                   row_idx: torch.Tensor | None = None, write_residual: bool = True,
                   out: torch.Tensor | None = None) -> torch.Tensor:
    """residual[src] += bf16(sum_s part[s, src] + bias); y[i] = layernorm(residual[src])."""
    S, Mpad, d = part.shape
    rows = row_idx.numel() if row_idx is not None else Mpad
    if not _gpu(part):
        return ref.slab_layernorm(part, residual, w, b, eps, bias, row_idx, write_residual)
    assert part.dtype == torch.float32 and part.is_contiguous()
    _bf16_contig(residual, "residual")
    assert residual.shape[-1] == d and residual.shape[0] >= Mpad
    if row_idx is not None:
        assert row_idx.dtype == torch.int64 and row_idx.is_contiguous()
    if bias is not None:
        _bf16_contig(bias, "bias")
        assert bias.numel() == d
    y = out if out is not None else torch.empty(rows, d, dtype=torch.bfloat16, device=part.device)
    check(kernels().loqa_slab_layernorm(ptr(part), S, Mpad, ptr(row_idx), rows, ptr(bias),
                                        ptr(residual), int(write_residual), ptr(w), ptr(b), ptr(y),
                                        d, eps, stream_ptr(part)), "slab_layernorm")
    return y


def slab_bias_act(part: torch.Tensor, bias: torch.Tensor | None, act: str = "none") -> torch.Tensor:
    """bf16(act(sum_s part + bias)) [Mpad, N]; act in {"none", "gelu"}."""
    S, Mpad, N = part.shape
    a = {"none": 0, "gelu": 1}[act]
    if not _gpu(part):
        return ref.slab_bias_act(part, bias, act)
    if bias is not None:
        _bf16_contig(bias, "bias")
        assert bias.numel() == N
    out = torch.empty(Mpad, N, dtype=torch.bfloat16, device=part.device)
    check(kernels().loqa_slab_bias_act(ptr(part), S, Mpad, Mpad, N, ptr(bias), a, ptr(out),
                                       stream_ptr(part)), "slab_bias_act")
    return out


def embed_pos(tokens: torch.Tensor, positions: torch.Tensor, tok_embed: torch.Tensor,
              pos_embed: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """bf16(tok_embed[tokens] + pos_embed[positions]) [rows, d]."""
    rows, d = tokens.numel(), tok_embed.shape[1]
    if not _gpu(tok_embed):
        return (tok_embed[tokens.long()].float() + pos_embed[positions.long()].float()).to(
            torch.bfloat16)
    assert tokens.dtype == torch.int32 and positions.dtype == torch.int32
    out = out if out is not None else torch.empty(rows, d, dtype=torch.bfloat16,
                                                  device=tok_embed.device)
    check(kernels().loqa_embed_pos(ptr(tokens), ptr(positions), ptr(tok_embed), ptr(pos_embed),
                                   ptr(out), rows, d, stream_ptr(tok_embed)), "embed_pos")
    return out


def embed_stats(tokens: torch.Tensor, tok_embed: torch.Tensor, scratch: "FusedScratch",
                positions: torch.Tensor | None = None, pos_embed: torch.Tensor | None = None,
                sums: bool = False) -> torch.Tensor:
    """Decode-step input of the fused-GEMM path in one launch: the embedded rows
    tok_embed[tokens] (+ pos_embed[positions]) [rows, d] bf16, with their row
    sums of squares (and sums) written to ``scratch`` as ONE partial tile for
    layer 0's norm prologue (what ``scratch.seed_stats`` computes)."""
    rows, d = tokens.numel(), tok_embed.shape[1]
    if not _gpu(tok_embed):
        x = tok_embed[tokens.long()]
        if pos_embed is not None:
            x = (x.float() + pos_embed[positions.long()].float()).to(torch.bfloat16)
        scratch.seed_stats(x, sums=sums)
        return x
    assert tokens.dtype == torch.int32 and tokens.is_contiguous()
    _bf16_contig(tok_embed, "tok_embed")
    if pos_embed is not None:
        assert positions is not None and positions.dtype == torch.int32
        assert positions.numel() == rows and positions.is_contiguous()
        _bf16_contig(pos_embed, "pos_embed")
        assert pos_embed.shape[1] == d
    assert rows <= scratch.rowsq.numel()
    out = torch.empty(rows, d, dtype=torch.bfloat16, device=tok_embed.device)
    check(kernels().loqa_embed_stats(ptr(tokens), ptr(positions if pos_embed is not None else None),
                                     ptr(tok_embed), ptr(pos_embed), ptr(out), ptr(scratch.rowsq),
                                     ptr(scratch.rowsum) if sums else None, rows, d,
                                     stream_ptr(tok_embed)), "embed_stats")
    scratch.stat_tiles = 1
    return out


def slab_silu_mul(part: torch.Tensor) -> torch.Tensor:
    S, Mpad, F2 = part.shape
    F = F2 // 2
    if not _gpu(part):
        return ref.slab_silu_mul(part)
    out = torch.empty(Mpad, F, dtype=torch.bfloat16, device=part.device)
    check(kernels().loqa_slab_silu_mul(ptr(part), S, Mpad, Mpad, F, ptr(out), stream_ptr(part)),
          "slab_silu_mul")
    return out


def slab_reduce(part: torch.Tensor) -> torch.Tensor:
    S, Mpad, N = part.shape
    if S == 1:
        return part[0]
    if not _gpu(part):
        return part.sum(0)
    out = torch.empty(Mpad, N, dtype=torch.float32, device=part.device)
    check(kernels().loqa_slab_reduce(ptr(part), S, Mpad, Mpad, N, ptr(out), stream_ptr(part)),
          "slab_reduce")
    return out


# ------------------------------------------------------------- VITS / HiFi-GAN
class ConvWeight:
    """A conv1d weight prepared for the MFMA implicit-GEMM kernel: [Cout_pad, K,
    Cin] bf16 (Cout padded to 32; gated convs interleave the tanh / sigmoid
    halves in 16-channel blocks). Keeps the torch-layout copy for the CPU path."""

    def __init__(self, w: torch.Tensor, bias: torch.Tensor | None = None, gated: bool = False):
        self.w, self.bias, self.gated = w, bias, gated      # w [Cout, Cin, K]
        Cout, Cin, K = w.shape
        self.Cout, self.Cin, self.K = Cout, Cin, K
        assert Cin % 16 == 0, "input channels must be a multiple of 16"
        perm = torch.arange(Cout, device=w.device)
        if gated:
            Hh = Cout // 2
            assert Hh % 16 == 0
            blocks = []
            for q in range(Hh // 16):
                blocks += [torch.arange(16 * q, 16 * q + 16), torch.arange(Hh + 16 * q, Hh + 16 * q + 16)]
            perm = torch.cat(blocks).to(w.device)
        cpad = (Cout + 31) // 32 * 32
        wp = torch.zeros(cpad, K, Cin, dtype=torch.bfloat16, device=w.device)
        wp[:Cout] = w[perm].permute(0, 2, 1).to(torch.bfloat16)
        self.wp = wp.contiguous()
        self.bp = None
        if bias is not None:
            bp = torch.zeros(cpad, dtype=torch.bfloat16, device=w.device)
            bp[:Cout] = bias[perm].to(torch.bfloat16)
            self.bp = bp
        self.cpad = cpad

    @property
    def out_channels(self) -> int:
        return self.Cout // 2 if self.gated else self.Cout


def conv1d(x: torch.Tensor, cw: ConvWeight, *, dil: int = 1, pad: int | None = None,
           stride: int = 1, pre_slope: float | None = None, act: str | None = None,
           res: torch.Tensor | None = None, alpha: float = 1.0, acc: torch.Tensor | None = None,
           lens: torch.Tensor | None = None, out: torch.Tensor | None = None,
           pcm16: bool = False, Tout: int | None = None, ostride: int = 1, ophase: int = 0,
           Tq: int | None = None) -> torch.Tensor:
    """Channels-last conv1d [B, Tin, Cin] -> [B, Tout, Cout'] with fused
    pre-activation (leaky ReLU), bias, act (relu / tanh / gated), residual add,
    scale, accumulate and length mask (see conv1d.hip). ``pad`` defaults to
    'same'. ``res``/``acc``/``out`` may be strided views; ``acc`` may alias ``out``."""
    B, Tin, Cin = x.shape
    assert Cin == cw.Cin
    if pad is None:
        pad = dil * (cw.K - 1) // 2
    if Tq is None:
        Tq = (Tin + 2 * pad - dil * (cw.K - 1) - 1) // stride + 1
    T_out = Tout if Tout is not None else Tq * ostride + ophase
    Co = cw.out_channels
    act_id = {None: 0, "relu": 1, "tanh": 2, "gated": 3}[act]
    assert (act == "gated") == cw.gated
    if not _gpu(x):
        y = ref.conv1d(x, cw.w, cw.bias, dil=dil, pad=pad, stride=stride, pre_slope=pre_slope,
                       act=act, res=res, alpha=alpha, acc=acc, lens=lens, Tout=T_out,
                       ostride=ostride, ophase=ophase, Tq=Tq)
        if pcm16:
            y = (y.clamp(-1, 1) * 32767).round().to(torch.int16)
        else:
            y = y.to(torch.bfloat16)
        if out is not None:
            if ostride == 1 and ophase == 0 and Tq == T_out:
                out.copy_(y)
            else:  # polyphase: only this phase's rows
                q = torch.arange(Tq, device=x.device) * ostride + ophase
                q = q[(q >= 0) & (q < T_out)]
                out[:, q] = y[:, q]
            return out
        return y
    assert x.dtype == torch.bfloat16 and x.stride(-1) == 1
    dt = torch.int16 if pcm16 else torch.bfloat16
    if out is None:
        out = torch.empty(B, T_out, Co, dtype=dt, device=x.device)
    assert out.dtype == dt and out.stride(-1) == 1 and out.shape[1] == T_out

    def bs(t):
        return (0, 0) if t is None else (t.stride(0), t.stride(1))
    for t in (res, acc):
        if t is not None:
            assert t.dtype == torch.bfloat16 and t.stride(-1) == 1 and t.shape[1] >= T_out
    if lens is not None:
        assert lens.dtype == torch.int32 and lens.numel() == B
    check(kernels().loqa_conv1d(
        ptr(x), x.stride(0), x.stride(1), ptr(cw.wp), ptr(cw.bp), ptr(out), out.stride(0),
        out.stride(1), ptr(res), *bs(res), ptr(acc), *bs(acc), ptr(lens), B, Tin, Cin, Tq,
        cw.cpad, cw.K, dil, pad, stride, ostride, ophase, T_out,
        0 if pre_slope is None else 1, float(pre_slope or 0.0), act_id, float(alpha), int(pcm16),
        Co, stream_ptr(x)), "conv1d")
    return out


class ConvTransposeWeight:
    """ConvTranspose1d(kernel Kt = 2s-style, stride s) as s polyphase convs:
    y[q*s + r - p] = sum_j x[q - j] w[:, :, r + j*s]."""

    def __init__(self, w: torch.Tensor, bias: torch.Tensor | None, stride: int, padding: int):
        Cin, Cout, Kt = w.shape
        assert Kt % stride == 0
        self.w, self.bias, self.stride, self.padding = w, bias, stride, padding
        self.taps = Kt // stride
        self.phases = []
        for r in range(stride):
            # tap kk of the regular conv reads x[q - (taps-1) + kk] with weight w[r + (taps-1-kk)*s]
            ks = [r + (self.taps - 1 - kk) * stride for kk in range(self.taps)]
            wr = w[:, :, ks].permute(1, 0, 2).contiguous()  # [Cout, Cin, taps]
            self.phases.append(ConvWeight(wr, bias))
        self.Cout = Cout

    def out_len(self, Tin: int) -> int:
        return (Tin - 1) * self.stride - 2 * self.padding + self.taps * self.stride


def conv_transpose1d(x: torch.Tensor, ct: ConvTransposeWeight, *,
                     pre_slope: float | None = None, polyphase: bool | None = None) -> torch.Tensor:
    """ConvTranspose1d on channels-last rows; on the GPU always as polyphase
    MFMA convolutions (``polyphase=True`` forces that decomposition on the CPU
    too, for testing)."""
    B, Tin, _ = x.shape
    T_out = ct.out_len(Tin)
    s, p = ct.stride, ct.padding
    if not _gpu(x) and not polyphase:
        return ref.conv_transpose1d(x, ct.w, ct.bias, stride=s, padding=p,
                                    pre_slope=pre_slope).to(torch.bfloat16)
    out = torch.zeros(B, T_out, ct.Cout, dtype=torch.bfloat16, device=x.device)
    for r, cw in enumerate(ct.phases):
        Tq = (T_out - r + p + s - 1) // s
        conv1d(x, cw, dil=1, pad=ct.taps - 1, stride=1, pre_slope=pre_slope, out=out, Tout=T_out,
               ostride=s, ophase=r - p, Tq=Tq)
    return out


def relpos_attention(qkv: torch.Tensor, emb_k: torch.Tensor, emb_v: torch.Tensor,
                     lens: torch.Tensor | None, n_heads: int, head_dim: int, window: int,
                     scale: float | None = None) -> torch.Tensor:
    """VITS windowed relative-position self-attention over q|k|v rows [B, T, 3C]."""
    B, T, _ = qkv.shape
    scale = scale if scale is not None else 1.0 / math.sqrt(head_dim)
    if not _gpu(qkv):
        return ref.relpos_attention(qkv, emb_k, emb_v, lens, n_heads, head_dim, window,
                                    scale).to(torch.bfloat16)
    assert qkv.dtype == torch.bfloat16 and qkv.stride(-1) == 1
    out = torch.empty(B, T, n_heads * head_dim, dtype=torch.bfloat16, device=qkv.device)
    check(kernels().loqa_relpos_attention(ptr(qkv), qkv.stride(1), ptr(emb_k), ptr(emb_v),
                                          ptr(lens), ptr(out), out.stride(1), B, T, n_heads,
                                          head_dim, window, scale, stream_ptr(qkv)),
          "relpos_attention")
    return out


def expand_sample(stats: torch.Tensor, cum: torch.Tensor, flen: torch.Tensor, F: int,
                  noise_scale: float, seed: int = 0,
                  seed_dev: torch.Tensor | None = None) -> torch.Tensor:
    """Length regulation + prior sampling: [B, T, 2C] stats -> z_p [B, F, C] bf16.
    ``seed_dev`` (GPU, int32 [1]): the seed read on the device (graph replay)."""
    B, T, C2 = stats.shape
    if not _gpu(stats):
        g = torch.Generator().manual_seed(seed)
        noise = torch.randn(B, F, C2 // 2, generator=g)
        return ref.expand_sample(stats, cum, flen, F, noise_scale, noise).to(torch.bfloat16)
    assert cum.dtype == torch.int32 and flen.dtype == torch.int32
    z = torch.empty(B, F, C2 // 2, dtype=torch.bfloat16, device=stats.device)
    check(kernels().loqa_expand_sample(ptr(stats), stats.stride(1), ptr(cum), B, T, ptr(flen),
                                       ptr(z), F, C2 // 2, float(noise_scale), seed & 0xFFFFFFFF,
                                       ptr(seed_dev), stream_ptr(stats)), "expand_sample")
    return z


# ------------------------------------------------------------ fused decode GEMMs
class FusedScratch:
    """Device state shared by the fused decode GEMMs of one engine: split-K
    ticket counters (zeroed once; each reducer resets its own) and the per-tile
    row statistics (sums of squares, sums) handed from the residual epilogues to
    the next GEMM's norm prologue."""

    def __init__(self, device, max_tiles: int = 8192, max_rows: int = 128):
        # max_rows = the largest Mpad (128): the 70B gate|up at Mpad 128 has
        # 3584 row tiles x 128 rows of statistics
        self.counters = torch.zeros(max_tiles, dtype=torch.int32, device=device)
        self.rowsq = torch.zeros(max_tiles * max_rows, dtype=torch.float32, device=device)
        self.rowsum = torch.zeros(max_tiles * max_rows, dtype=torch.float32, device=device)
        self.stat_tiles = 0   # partial tiles written by the last residual epilogue
        # ticket / item counters of the prologue-item launches (skinny_fused
        # ``prologue``): zero between launches, each launch resets its own
        self.pro_ctr = torch.zeros(2, dtype=torch.int32, device=device)

    def seed_stats(self, x: torch.Tensor, sums: bool = True) -> None:
        """Row statistics of ``x`` as ONE partial tile (layer 0's norm input)."""
        M = x.shape[0]
        xf = x.float()
        torch.sum(xf.square(), 1, out=self.rowsq[:M])
        if sums:
            torch.sum(xf, 1, out=self.rowsum[:M])
        self.stat_tiles = 1


_FUSED_MODES = {"silu": 1, "resid": 2, "rope": 3, "act": 4}
_NORMS = {None: 0, False: 0, True: 1, "rms": 1, "ln": 2}
_ACTS = {"none": 0, "gelu": 1, "f32": 2}   # "f32": no activation, f32 output


class FusedLinear:
    """A decode projection prepared for the fused GEMM: the pre-shuffled weight
    (rows optionally permuted), with the input norm's weight folded into it and
    the norm's shift / the linear bias folded into one f32 output bias.

    norm "rms": rmsnorm(x; g) W^T            -> s * (W g) x
    norm "ln" : layernorm(x; g, b) W^T + c   -> s * ((W g) x - mean * colsum) + (W b + c)
    """

    def __init__(self, w: torch.Tensor, *, norm: str | None = None, norm_w=None, norm_b=None,
                 bias=None, perm: torch.Tensor | None = None):
        wf = w.float()
        self.norm = norm
        if norm is not None:
            wf = wf * norm_w.float()[None, :]
        wb = wf.to(torch.bfloat16)
        b = torch.zeros(w.shape[0], dtype=torch.float32, device=w.device)
        if bias is not None:
            b = b + bias.float()
        if norm == "ln" and norm_b is not None:
            # W @ beta as a multiply + row sum (load time; keeps rocBLAS's GEMV
            # out of the process, so a kernel trace holds no vendor BLAS at all)
            b = b + (w.float() * norm_b.float()[None, :]).sum(1)
        self.colsum = wb.float().sum(1) if norm == "ln" else None
        self.has_bias = bias is not None or (norm == "ln" and norm_b is not None)
        if perm is not None:
            wb = wb[perm]
            b = b[perm]
            if self.colsum is not None:
                self.colsum = self.colsum[perm].contiguous()
        self.bias = b.contiguous() if self.has_bias else None
        self.wp = shuffle_weight(wb.contiguous())
        self.N, self.K = w.shape


def tune_fused(wp, mode: str, *, mpads=(16, 32, 64, 128), norm=None, act: str = "none",
               heads: tuple | None = None, cos_sin=None, prefill: bool = False,
               xl: bool = True, pro_compat: bool = False) -> None:
    """Measure the split-K of one fused decode GEMM shape on dummy operands
    (``heads`` = (H, Hkv, D) for "rope"); before any graph capture.
    ``pro_compat``: at Mpad 16 / 32 only the layouts a prologue launch runs
    (4 waves along K, 4-step prefetch groups), so a tensor-parallel step with
    and without prologues computes in the same order (bitwise equal).
    ``prefill``: Mpad 64 is the chunked prefill of compact weights (a whole
    weight pass per 64 tokens, on its own stream): 64-row tiles and 4 waves
    along rows are then candidates too (70B gate|up 64 tokens: 204 us vs 483 us
    for 16-row tiles). Otherwise Mpad 64 is a decode step beside the Whisper
    decoder, where those long-lived workgroups slow the pipeline."""
    lin = wp if isinstance(wp, FusedLinear) else None
    w = lin.wp if lin is not None else wp
    if not _gpu(w) or NO_TUNE:
        return
    dev = w.device
    N, K = w.shape[0] * 16, w.shape[1] * 32
    scr = FusedScratch(dev)
    bf = dict(dtype=torch.bfloat16, device=dev)
    nrm = norm if norm is not None else (lin.norm if lin is not None else None)
    # cold-weight timing: enough copies that the set outgrows the Infinity Cache
    nbytes = w.numel() * w.element_size()
    copies = [wp]
    for _ in range(min(15, -(-(768 << 20) // nbytes) - 1)):
        if lin is not None:
            c = copy.copy(lin)
            c.wp = lin.wp.clone()
        else:
            c = wp.clone()
        copies.append(c)
    xl_on = xl and os.environ.get("LOQA_TUNE_XL", "1") != "0"
    for Mpad in mpads:
        if Mpad == 128 and not xl_on:
            continue
        key = (mode, N, K, Mpad)
        if key in _FSPLITS:
            continue
        x = torch.randn(Mpad, K, **bf)
        kw: dict = {}
        if nrm:
            tiles = max(1, K // 32)
            scr.rowsq[: tiles * Mpad].fill_(float(K) / tiles)
            kw.update(rowsq_tiles=tiles)
        if mode == "resid":
            kw.update(residual=torch.zeros(Mpad, N, **bf))
        elif mode == "act":
            kw.update(act=act)
        elif mode == "rope":
            H, Hkv, D = heads
            kc = torch.zeros(max(4, Mpad // 16), Hkv, 16, D, **bf)   # one slot per row
            pos = torch.arange(Mpad, dtype=torch.int32, device=dev)
            kw.update(positions=pos, cos_sin=cos_sin, q_out=torch.empty(Mpad, H * D, **bf),
                      k_cache=kc, v_cache=torch.zeros_like(kc), slots=pos, n_heads=H, n_kv=Hkv,
                      head_dim=D)
        wide = Mpad <= 32 or prefill
        rts = (1, 2, 4) if (prefill and Mpad == 64) else (1, 2)
        # XL layouts only at Mpad 128: at Mpad 64 / 32 they win in isolation but,
        # as decode steps beside the Whisper decoder, took the pipeline from 17.6
        # to 10.3 utt/s (long-lived 4-wave workgroups: the co-scheduling cliff,
        # docs/PERF.md)
        xl = "only" if Mpad == 128 else "no"
        pc = pro_compat and Mpad in (16, 32)
        tune_fused_splits(key, lambda sp, rt, wr, i, xl_=0: skinny_fused(
            x, copies[i], mode, scr, splits=sp, rt=rt, wr=wr, norm=nrm, xl=xl_, **kw), K, rts=rts,
            ncopies=len(copies), wr4=wide and not pc, fewest=wide, xl=xl,
            splits=[sp for sp in SPLIT_CANDIDATES if (K // 32 // (sp * 4)) % 4 == 0] if pc else None)
    del copies


def fold_norm(w: torch.Tensor, norm_w: torch.Tensor) -> torch.Tensor:
    """Weight rows with an RMSNorm weight folded in (W * diag(g)), the operand
    of a ``norm=True`` fused GEMM: rmsnorm(x) W^T = s(x) * (x (W diag(g))^T)."""
    return (w.float() * norm_w.float()[None, :]).to(w.dtype)


def skinny_fused(x: torch.Tensor, wp, mode: str, scratch: FusedScratch, *,
                 splits: int | None = None, norm=None, eps: float = 1e-5,
                 rowsq_tiles: int | None = None, rt: int | None = None,
                 residual: torch.Tensor | None = None, positions=None, cos_sin=None, q_out=None,
                 k_cache=None, v_cache=None, slots=None, n_heads: int = 0, n_kv: int = 0,
                 head_dim: int = 0, out=None, act: str = "none", bias=None, colsum=None,
                 row_sums: bool = False, wr: int | None = None, xl: int | None = None,
                 attn: dict | None = None, prologue: dict | None = None) -> torch.Tensor:
    """Skinny GEMM with a fused epilogue and optional input norm; Mpad 16, 32,
    64 or 128 (``xl``: activations staged through LDS, 4 waves along rows,
    required at Mpad 128; chosen by the tuner at 64).

    ``wp`` is a shuffled weight or a ``FusedLinear`` (which supplies the norm
    kind unless ``norm`` is given, the folded bias and the LayerNorm column
    sums). ``norm`` True/"rms":
    RMSNorm, "ln": LayerNorm; the row statistics come from ``rowsq_tiles``
    partial tiles in ``scratch`` (default: what the last residual epilogue wrote); the norm
    weight is folded into the weight.
    mode "silu": returns bf16 [Mpad, N/2] (weights in ``perm_gate_up`` order);
    "resid": residual += x W^T (+ bias) in place, writes per-tile row sums of
    squares (and row sums with ``row_sums``);
    "rope": q -> q_out, k (RoPE'd when ``cos_sin``) and v -> paged caches
    (``perm_rope_qkv`` order); "act": returns act(x W^T + bias) bf16 [Mpad, N].

    ``attn`` (mode "rope"): the step's causal decode attention over the paged
    caches (keys of :func:`attention`: cu_q, ctx_lens, block_tables, max_q,
    split_keys, num_splits, workspace, max_k, scale, out) follows the GEMM and
    its output is returned (mode "act": attention over contiguous K / V rows,
    keys k, v, kv_start). Two launches: the one-launch hand-off was measured
    slower in every configuration and removed (docs/PERF.md, round 5).

    ``prologue``: the short step that produces x runs INSIDE this launch
    (gemm_skinny.hip PRO; the weight stream starts at once, the tiles read x
    after every item is done). ``dict(kind="car", car=<CustomAllReduce>,
    which=0|1, nblk=n)``: the tensor-parallel residual all-reduce of input
    buffer ``which`` - x is the residual it updates in place, its world x nblk
    statistics tiles are this GEMM's norm input (mode "silu" / "rope", RMSNorm).
    ``dict(kind="attn", q=, k_cache=, v_cache=, cu_q=, ctx_lens=,
    block_tables=, n_heads=, n_kv=, max_q=, split_keys=, num_splits=,
    workspace=, scale=)``: paged causal decode attention whose output is x
    (D = 128; mode "act" / "resid"). ``pro_wgs`` in the dict caps the grid
    (the one-GPU multi-rank rehearsal)."""
    if attn is not None:
        assert mode in ("rope", "act")
        rope = mode == "rope"
        if not rope and out is None:
            out = torch.empty(x.shape[0], wp.shape[0] * 16 if not isinstance(wp, FusedLinear)
                              else wp.N, dtype=torch.bfloat16, device=x.device)
        qq = skinny_fused(x, wp, mode, scratch, splits=splits, norm=norm, eps=eps,
                          rowsq_tiles=rowsq_tiles, rt=rt, positions=positions, cos_sin=cos_sin,
                          q_out=q_out, k_cache=k_cache, v_cache=v_cache, slots=slots,
                          n_heads=n_heads, n_kv=n_kv, head_dim=head_dim, bias=bias,
                          colsum=colsum, wr=wr, xl=xl, out=out, act=act)
        if rope:
            return attention(q_out, k_cache, v_cache, attn["cu_q"], n_heads=n_heads,
                             n_kv=n_kv, head_dim=head_dim, causal=True, max_q=attn["max_q"],
                             ctx_lens=attn["ctx_lens"], block_tables=attn["block_tables"],
                             scale=attn.get("scale"), grouped=True,
                             split_keys=attn["split_keys"], num_splits=attn["num_splits"],
                             workspace=attn["workspace"], out=attn.get("out"),
                             max_k=attn.get("max_k"))
        return attention(qq, attn["k"], attn["v"], attn["cu_q"], n_heads=n_heads, n_kv=n_kv,
                         head_dim=head_dim, causal=False, max_q=attn["max_q"],
                         cu_k=attn["kv_start"], ctx_lens=attn["ctx_lens"],
                         scale=attn.get("scale"), grouped=True,
                         split_keys=attn["split_keys"], num_splits=attn["num_splits"],
                         workspace=attn["workspace"], out=attn.get("out"))
    if isinstance(wp, FusedLinear):
        lin = wp
        wp = lin.wp
        norm = lin.norm if norm is None else norm
        bias = lin.bias if bias is None else bias
        colsum = lin.colsum if colsum is None else colsum
    Mpad, K = x.shape
    N = wp.shape[0] * 16
    nrm = _NORMS[norm]
    tuned = _FSPLITS.get((mode, N, K, Mpad))
    S = splits or (tuned[0] if tuned else choose_splits(N, K, Mpad))
    rt = rt or (tuned[1] if tuned else (1 if Mpad == 128 else 2))
    if xl is None:
        xl = tuned[3] if (tuned and not splits and len(tuned) > 3) else int(Mpad == 128)
    if wr is None:
        wr = tuned[2] if (tuned and not splits and len(tuned) > 2) else 1
    if xl:
        wr = 4
        rt = rt if rt in (1, 2) and N % (64 * rt) == 0 else 1
    elif wr != 1 and (S != 1 or N % (64 * rt)):
        wr = 1
    if rowsq_tiles is None:
        rowsq_tiles = scratch.stat_tiles
    m = _FUSED_MODES[mode]
    ntiles = N // (16 * rt)
    if mode == "resid":
        scratch.stat_tiles = ntiles
    if mode == "silu" and out is None:
        out = torch.empty(Mpad, N // 2, dtype=torch.bfloat16, device=x.device)
    elif mode == "act" and out is None:
        out = torch.empty(Mpad, N, dtype=torch.float32 if act == "f32" else torch.bfloat16,
                          device=x.device)
    if not _gpu(x):
        return _skinny_fused_ref(x, wp, mode, scratch, nrm, eps, rowsq_tiles, residual,
                                 positions, cos_sin, q_out, k_cache, v_cache, slots, n_heads,
                                 n_kv, head_dim, out, act, bias, colsum, row_sums, rt)
    assert Mpad in (16, 32, 64, 128) and x.dtype == torch.bfloat16 and x.stride(1) == 1
    assert Mpad != 128 or xl, "Mpad 128 needs the XL layout"
    assert ntiles <= scratch.counters.numel() and ntiles * Mpad <= scratch.rowsq.numel()
    if nrm == 2:
        assert colsum is not None and colsum.numel() == N
    if bias is not None:
        assert bias.dtype == torch.float32 and bias.numel() == N and bias.is_contiguous()
    if mode == "act":
        assert out.dtype == (torch.float32 if act == "f32" else torch.bfloat16)
        assert out.stride(0) % 4 == 0 and out.shape[0] >= Mpad and out.shape[1] >= N
    if mode == "rope":   # the epilogue reads slots / positions for every padded row
        assert slots.numel() >= Mpad and q_out.shape[0] >= Mpad and k_cache.is_contiguous()
        assert cos_sin is None or positions.numel() >= Mpad
    elif mode == "resid":
        assert residual.shape[0] >= Mpad and residual.shape[1] == N
    part = torch.empty(S, Mpad, N, dtype=torch.float32, device=x.device) if S > 1 else None
    blk = k_cache.shape[2] if k_cache is not None else 0
    if prologue is not None and not (wr == 1 and not xl and Mpad in (16, 32) and rt in (1, 2)
                                     and (K // 32 // (S * 4)) % 4 == 0):
        # a layout the prologue launch form (4 waves along K, no XL, Mpad 16 /
        # 32, 4-step prefetch groups) does not run: the prologue as its own
        # kernel first - the same arithmetic, one more launch
        _prologue_standalone(prologue, x, scratch)
        prologue = None
    p = FusedParams()
    p.x, p.ldx, p.Wp, p.part, p.counters = ptr(x), x.stride(0), ptr(wp), ptr(part), \
        ptr(scratch.counters)
    p.Mpad, p.N, p.K, p.S, p.mode, p.norm = Mpad, N, K, S, m, nrm
    if nrm:
        p.rowsq_in, p.rowsum_in = ptr(scratch.rowsq), ptr(scratch.rowsum)
    p.rowstat_tiles, p.eps = rowsq_tiles, eps
    p.colsum, p.bias = ptr(colsum), ptr(bias)
    p.out, p.ldo, p.act = ptr(out), (out.stride(0) if out is not None else 0), _ACTS[act]
    if mode == "resid":
        p.residual, p.rowsq_out = ptr(residual), ptr(scratch.rowsq)
        p.rowsum_out = ptr(scratch.rowsum) if row_sums else None
    p.positions, p.cs, p.q_out = ptr(positions), ptr(cos_sin), ptr(q_out)
    p.kc, p.vc, p.slots = ptr(k_cache), ptr(v_cache), ptr(slots)
    p.H, p.Hkv, p.D, p.blk = n_heads, n_kv, head_dim, blk
    p.rt, p.wr, p.xl = rt, wr, int(bool(xl))
    if prologue is not None:
        _set_prologue(p, prologue, x, scratch, Mpad, K, rowsq_tiles)
    check(kernels().loqa_skinny_fused(ctypes.byref(p), stream_ptr(x)), "skinny_fused")
    if mode in ("silu", "act"):
        return out
    return q_out if mode == "rope" else residual


def set_launch_priority(prio: int) -> None:
    """Wave issue priority (s_setprio 3) of the decode attention and fused
    GEMM kernels this host THREAD launches or captures from now on (0 =
    default); the STT decoder thread sets it under ``LOQA_STT_WAVE_PRIO``."""
    if torch.cuda.is_available():
        kernels().loqa_set_launch_prio(int(prio))


PRO_KINDS = {"car": 1, "attn": 2}


def _prologue_standalone(pro: dict, x, scratch) -> None:
    """The prologue of a skinny_fused launch as its own kernel (same numerics)."""
    if pro["kind"] == "car":
        pro["car"].resid(pro["which"], x, scratch.rowsq, pro["nblk"])
        return
    attention(pro["q"], pro["k_cache"], pro["v_cache"], pro["cu_q"], n_heads=pro["n_heads"],
              n_kv=pro["n_kv"], head_dim=pro["k_cache"].shape[3], causal=True, max_q=pro["max_q"],
              ctx_lens=pro["ctx_lens"], block_tables=pro["block_tables"], scale=pro.get("scale"),
              grouped=True, split_keys=pro["split_keys"], num_splits=pro["num_splits"],
              workspace=pro["workspace"], out=x, max_k=pro.get("max_k"))
# tensor-parallel decode steps with the all-reduces / attention as GEMM
# prologues (models/llama.py _decode_fused_tp_prologue; grid cap:
# CustomAllReduce.prologue_wgs). Off by default: 328 instead of 567 launches
# per config-5 rank step, bitwise the same logits, but 7.86 vs 6.87 ms per
# step (profiles/r6_config5_prologue_ab.txt, docs/PERF.md round 6)
TP_PROLOGUE = os.environ.get("LOQA_TP_PROLOGUE", "0") == "1"


def _set_prologue(p, pro: dict, x, scratch, Mpad: int, K: int, rowsq_tiles: int) -> None:
    kind = PRO_KINDS[pro["kind"]]
    assert Mpad in (16, 32), "prologue launches: Mpad 16 / 32"
    p.pro, p.pro_ctr, p.pro_wgs = kind, ptr(scratch.pro_ctr), int(pro.get("pro_wgs", 0))
    if kind == 1:
        car = pro["car"]
        assert x.stride(0) == K and rowsq_tiles == car.world * pro["nblk"]
        p.car, p.car_which, p.car_nblk = car._h, int(pro["which"]), int(pro["nblk"])
        return
    q, kc, vc, ws = pro["q"], pro["k_cache"], pro["v_cache"], pro["workspace"]
    H, Hkv = pro["n_heads"], pro["n_kv"]
    D = kc.shape[3]
    B = pro["cu_q"].numel() - 1
    assert D == 128 and H * D == K and (H // Hkv) * pro["max_q"] <= 32
    assert pro["split_keys"] % 32 == 0 and ws.max_splits >= pro["num_splits"]
    assert ws.max_tokens >= q.shape[0] and B * Hkv <= ws.counters.numel() and q.shape[0] <= Mpad
    bt = pro["block_tables"]
    assert kc.is_contiguous() and vc.is_contiguous() and bt.is_contiguous()
    if pro.get("max_k") is not None:
        assert pro["max_k"] <= bt.shape[1] * kc.shape[2], "context exceeds block table"
    sc = pro.get("scale")
    p.att_q, p.att_q_stride, p.att_kc, p.att_vc = ptr(q), q.stride(0), ptr(kc), ptr(vc)
    p.att_cu_q, p.att_ctx, p.att_bt = ptr(pro["cu_q"]), ptr(pro["ctx_lens"]), ptr(bt)
    p.att_max_blocks, p.att_blk = bt.shape[1], kc.shape[2]
    p.att_B, p.att_Hq, p.att_Hkv = B, H, Hkv
    p.att_split_keys, p.att_num_splits, p.att_total_q = pro["split_keys"], pro["num_splits"], q.shape[0]
    p.att_scale = sc if sc is not None else 1.0 / math.sqrt(D)
    p.att_part_o, p.att_part_ml, p.att_counters = ptr(ws.part_o), ptr(ws.part_ml), ptr(ws.counters)


def _skinny_fused_ref(x, wp, mode, scratch, nrm, eps, rowsq_tiles, residual, positions,
                      cos_sin, q_out, k_cache, v_cache, slots, H, Hkv, D, out, act, bias, colsum,
                      row_sums, rt=2):
    Mpad, K = x.shape
    N = wp.shape[0] * 16
    y = x.float() @ ref.unshuffle_weight(wp).float().t()  # [Mpad, N] in permuted row order
    if nrm:
        rs = scratch.rowsq[: rowsq_tiles * Mpad].view(rowsq_tiles, Mpad)
        if nrm == 1:
            y = y * ref.fused_row_scale(rs, eps, K)[:, None]
        else:
            sm = scratch.rowsum[: rowsq_tiles * Mpad].view(rowsq_tiles, Mpad)
            mean, rstd = ref.fused_ln_stats(rs, sm, eps, K)
            y = rstd[:, None] * (y - mean[:, None] * colsum.float()[None, :])
    if bias is not None:
        y = y + bias.float()[None, :]
    if mode == "silu":
        F = N // 2
        inv = torch.argsort(ref.perm_gate_up(F))
        y = y[:, inv]
        out.copy_(ref.silu_mul(y.to(torch.bfloat16)))
        return out
    if mode == "act":
        if act == "f32":
            out.copy_(y)
            return out
        yb = y.to(torch.bfloat16)
        if act == "gelu":
            yb = torch.nn.functional.gelu(yb.float()).to(torch.bfloat16)
        out.copy_(yb)
        return out
    if mode == "resid":
        h = (y + residual.float()).to(torch.bfloat16)
        residual.copy_(h)
        R = 16 * rt
        sq = h.float().pow(2).view(Mpad, N // R, R).sum(-1).t().contiguous()  # [tiles, Mpad]
        scratch.rowsq[: sq.numel()] = sq.flatten()
        if row_sums:
            sm = h.float().view(Mpad, N // R, R).sum(-1).t().contiguous()
            scratch.rowsum[: sm.numel()] = sm.flatten()
        return residual
    inv = torch.argsort(ref.perm_rope_qkv(H, Hkv, D))
    qkv = y[:, inv].to(torch.bfloat16)
    ref.rope_kv_append(qkv, positions, cos_sin, k_cache, v_cache, slots, H, Hkv, D)
    q_out.copy_(qkv[:, : H * D])
    return q_out


# ------------------------------------------------------------- prefill GEMM
PREFILL_GEMM_NT = 128     # features per workgroup of the default layout (3)


# v2 layouts: (row tiles, feature tiles) per wave and waves along M (the other
# 4 / WM waves go along N) -> workgroup tile (16 WM rbw) x (16 (4 / WM) ft)
PREFILL2_LAYOUTS = {0: (5, 4, 2), 1: (10, 4, 2), 2: (5, 2, 2), 3: (10, 2, 1), 4: (10, 4, 1)}
# layout 3 (v1's 1 x 4 waves with the one-barrier pipeline) measured fastest on
# every prefill / encoder shape (profiles/r3_prefill_gemm2_layouts.txt)
PREFILL2_LAYOUT = 3


def prefill_gemm2(x: torch.Tensor, wp: torch.Tensor, splits: int = 1, epi: str = "bf16",
                  layout: int | None = None) -> torch.Tensor:
    """x [M, K] bf16 @ W^T for prefill-sized M (64 - a few thousand rows), W
    pre-shuffled (``shuffle_weight``; ``csrc/kernels/gemm_prefill.hip`` v2).
    ``epi``: "bf16" -> [M, N]; "slabs" -> f32 split-K partials [S, M, N] (a
    slab consumer sums them); "swiglu" -> silu(gate) * up [M, N / 2] bf16 from
    a ``perm_gate_up`` weight (16-row gate|up pair tiles)."""
    M, K = x.shape
    N = wp.shape[0] * 16
    assert wp.shape[1] * 32 == K
    lay = PREFILL2_LAYOUT if layout is None else layout
    rbw, ft, wm = PREFILL2_LAYOUTS[lay]
    e = {"bf16": 0, "slabs": 1, "swiglu": 2}[epi]
    assert e == 1 or splits == 1
    if not _gpu(x):
        part = ref.skinny_gemm(x, wp, splits)
        if e == 1:
            return part
        y = part.sum(0)
        if e == 2:
            y = ref.swiglu_pairs(y)
        return y.to(torch.bfloat16)
    _bf16_contig(x, "x")
    assert N % (16 * ft * (4 // wm)) == 0 and K % (splits * 64) == 0, (N, K, splits, lay)
    if e == 1:
        out = torch.empty(splits, M, N, dtype=torch.float32, device=x.device)
        rc = kernels().loqa_gemm_prefill2(ptr(x), M, K, ptr(wp), N, splits, None, ptr(out), 1, lay,
                                          stream_ptr(x))
    else:
        out = torch.empty(M, N // 2 if e == 2 else N, dtype=torch.bfloat16, device=x.device)
        rc = kernels().loqa_gemm_prefill2(ptr(x), M, K, ptr(wp), N, 1, ptr(out), None, e, lay,
                                          stream_ptr(x))
    check(rc, "gemm_prefill2")
    return out


# ------------------------------------------------------- LDS-tiled MFMA GEMM
# csrc/kernels/gemm_tile.hip: (waves along N, waves along M, LDS stages); the
# workgroup tile is (64 * WN features) x (64 * WM rows).
GEMM_TILE_LAYOUTS = {0: (2, 2, 2), 1: (2, 2, 3), 2: (4, 2, 2), 3: (2, 4, 2), 4: (4, 2, 3),
                     5: (2, 4, 3), 6: (2, 4, 2), 7: (4, 2, 2), 8: (2, 2, 2), 9: (2, 2, 2)}
# (FN, FM) 16-wide MFMA fragments per wave along features / rows
GEMM_TILE_FRAGS = {6: (8, 4), 7: (4, 8), 8: (8, 4), 9: (4, 8)}


def gemm_tile_dims(layout: int) -> tuple[int, int]:
    """(features, rows) of a layout's workgroup tile."""
    wn, wm, _ = GEMM_TILE_LAYOUTS[layout]
    fn, fm = GEMM_TILE_FRAGS.get(layout, (4, 4))
    return 16 * fn * wn, 16 * fm * wm
_GT_EPI = {"bf16": 0, "slabs": 1, "swiglu": 2}
_GT_ZEROS: dict = {}


def gemm_tile_layout(M: int, N: int, K: int, epi: str = "bf16") -> int:
    """Layout for a shape: the measured best (layout 1 on every served shape,
    scripts/exp/gemm_tile_bench.py, docs/PERF.md); callers pass ``layout=``
    to force another."""
    return 1


def _gt_ref(x2: torch.Tensor, w: torch.Tensor, bias, act: str | None, pos, epi: str, splits: int):
    xf, wf = x2.float(), w.float()
    if epi == "slabs":
        K = xf.shape[1]
        ks = K // splits
        return torch.stack([xf[:, s * ks:(s + 1) * ks] @ wf[:, s * ks:(s + 1) * ks].t()
                            for s in range(splits)])
    y = xf @ wf.t()
    if epi == "swiglu":
        F = w.shape[0] // 2
        g = y[:, :F].to(torch.bfloat16).float()
        u = y[:, F:].to(torch.bfloat16).float()
        return (g * torch.sigmoid(g) * u).to(torch.bfloat16)
    if bias is not None:
        y = y + bias.float()
    if act == "gelu":
        y = y.to(torch.bfloat16).float()
        y = 0.5 * y * (1.0 + torch.erf(y * 0.70710678118654752))
    if pos is not None:
        rows = torch.arange(y.shape[0], device=y.device) % pos.shape[0]
        y = y.to(torch.bfloat16).float() + pos.float()[rows]
    return y.to(torch.bfloat16)


def conv_k3_weight(w: torch.Tensor, cin: int) -> torch.Tensor:
    """torch conv1d weight flattened [Cout, Cin * 3] (k = c * 3 + tap) -> the
    tiled GEMM's implicit-im2col order [Cout, 3 * Cin] (k = tap * Cin + c)."""
    cout = w.shape[0]
    return w.reshape(cout, cin, 3).permute(0, 2, 1).reshape(cout, 3 * cin).contiguous()


def conv_k3_im2col_ref(x: torch.Tensor, B: int, tin: int, stride: int) -> torch.Tensor:
    """Reference implicit im2col: x [B * tin, cin] time-major -> [B * tout, 3 * cin]
    (k = tap * cin + c, zero padding 1)."""
    cin = x.shape[1]
    xb = x.reshape(B, tin, cin)
    xp = torch.nn.functional.pad(xb, (0, 0, 1, 1))
    tout = (tin + 2 - 3) // stride + 1
    cols = [xp[:, tap: tap + stride * (tout - 1) + 1: stride] for tap in range(3)]
    return torch.cat(cols, dim=2).reshape(B * tout, 3 * cin)


def gemm_tile(x: torch.Tensor, w: torch.Tensor, *, bias: torch.Tensor | None = None,
              act: str | None = None, pos: torch.Tensor | None = None, epi: str = "bf16",
              splits: int = 1, layout: int | None = None, out: torch.Tensor | None = None,
              conv: tuple[int, int] | None = None) -> torch.Tensor:
    """Y = X W^T on the LDS-tiled MFMA GEMM (``csrc/kernels/gemm_tile.hip``).

    x [M, K] bf16 (row stride may exceed K), w [N, K] bf16 row-major.
    ``epi``: "bf16" -> [M, N] (+ f32 ``bias``, ``act`` "gelu", + bf16 ``pos``
    rows m % len(pos)); "slabs" -> f32 split-K partials [S, M, N]; "swiglu" ->
    silu(gate) * up [M, N / 2] with gate rows [0, N/2) and up rows [N/2, N).
    ``conv`` = (B, stride): x is a time-major conv input [B * T_in, Cin] and w a
    ``conv_k3_weight`` [N, 3 * Cin]; the output rows are (b, t_out) of the
    k = 3, padding 1 conv1d (implicit im2col: the input rows are gathered by the
    tile loader, no column matrix is built)."""
    N, K = w.shape
    if conv is not None:
        B, stride = conv
        cin = x.shape[1]
        assert K == 3 * cin
        tin = x.shape[0] // B
        tout = (tin + 2 - 3) // stride + 1
        M = B * tout
    else:
        M = x.shape[0]
        assert x.shape[1] == K, (x.shape, w.shape)
    if not _gpu(x):
        x2 = conv_k3_im2col_ref(x, B, tin, stride) if conv is not None else x
        y = _gt_ref(x2, w, bias, act, pos, epi, splits)
        if out is not None:
            out.copy_(y)
            return out
        return y
    if x.dtype != torch.bfloat16 or w.dtype != torch.bfloat16:
        raise TypeError("gemm_tile needs bf16 operands")
    if x.stride(1) != 1 or not w.is_contiguous():
        raise ValueError("gemm_tile needs K-contiguous operands")
    lay = gemm_tile_layout(M, N, K, epi) if layout is None else layout
    e = _GT_EPI[epi]
    p = _lib.GemmTileParams()
    p.x, p.ldx, p.w = ptr(x), x.stride(0), ptr(w)
    p.M, p.N, p.K, p.S, p.epi = M, N, K, splits, e
    p.act = 1 if act == "gelu" else 0
    if bias is not None:
        assert bias.dtype == torch.float32 and bias.is_contiguous() and bias.numel() == N
    p.bias = ptr(bias)
    if pos is not None:
        assert pos.dtype == torch.bfloat16 and pos.is_contiguous() and pos.shape[1] == N
        p.pos, p.pos_rows = ptr(pos), pos.shape[0]
    if e == 1:
        y = out if out is not None else torch.empty(splits, M, N, dtype=torch.float32,
                                                    device=x.device)
        p.part = ptr(y)
    else:
        cols = N // 2 if e == 2 else N
        y = out if out is not None else torch.empty(M, cols, dtype=torch.bfloat16, device=x.device)
        assert y.shape == (M, cols) and y.stride(1) == 1
        p.y, p.ldy = ptr(y), y.stride(0)
    if conv is not None:
        z = _GT_ZEROS.get((x.device, cin))
        if z is None:
            z = _GT_ZEROS[(x.device, cin)] = torch.zeros(max(cin, 64), dtype=torch.bfloat16,
                                                         device=x.device)
        p.conv_cin, p.conv_tin, p.conv_tout, p.conv_stride, p.zeros = cin, tin, tout, stride, ptr(z)
    p.layout = lay
    check(kernels().loqa_gemm_tile(ctypes.byref(p), stream_ptr(x)), "gemm_tile")
    return y


# ---------------------------------------------------------------------------
# Split-K tiled GEMM with an in-launch reduction (csrc/kernels/gemm_sk.hip)
_SK_EPI = {"bf16": 0, "swiglu": 1, "resid": 2}
# layout -> (features, rows, resident workgroups per CU (LDS), per-CU efficiency)
# efficiency: relative MFMA rate of the wave tile (LDS bytes per MFMA: 64 x 64
# = 1.0; 64 x 32 tiles read 1.5x the LDS per MFMA; 128 x 64 0.75x)
SK_LAYOUTS = {0: (128, 128, 2, 1.0), 1: (128, 64, 3, 0.85), 2: (256, 64, 2, 1.0),
              3: (256, 128, 1, 1.0), 4: (128, 64, 2, 0.9), 5: (128, 128, 1, 1.05),
              6: (256, 256, 1, 1.15), 7: (64, 64, 4, 0.6), 8: (256, 64, 1, 1.05),
              9: (256, 128, 1, 1.1), 10: (128, 128, 1, 1.1), 11: (128, 64, 1, 0.95)}
SK_CUS = 256
_SK_WS: dict = {}


# measured picks (scripts/exp/gemm_sk_bench.py --grid, cold weights, one
# MI355X; profiles/r4_gemm_sk_grid.txt): (N, K) -> [(max M, layout, chunks)]
SK_TABLE = {
    (6144, 4096): [(400, 4, 1), (900, 5, 1), (1 << 30, 0, 1)],        # Llama-3-8B qkv
    (4096, 4096): [(900, 4, 1), (1 << 30, 1, 1)],                     # o
    (28672, 4096): [(400, 4, 1), (1 << 30, 0, 1)],                    # gate|up
    (4096, 14336): [(400, 8, 3), (900, 0, 3), (1 << 30, 0, 1)],       # down
    (3840, 1280): [(1 << 30, 0, 1)],                                  # Whisper-large-v3 enc qkv
    (1280, 1280): [(2000, 4, 1), (4000, 5, 1), (1 << 30, 3, 1)],      # enc o
    (5120, 1280): [(1 << 30, 0, 1)],                                  # enc fc1
    (1280, 5120): [(2000, 4, 1), (4000, 5, 1), (1 << 30, 0, 1)],      # enc fc2
}


def gemm_sk_plan(M: int, N: int, K: int, epi: str = "bf16",
                 layouts=(0, 1, 2, 3, 4, 5)) -> tuple[int, int]:
    """(layout, K chunks) for a shape: the measured table for the served
    shapes, else an analytic plan - the fewest
    MFMA-cycle rounds over the resident workgroup slots, counting padded rows
    and wave-tile efficiency, with at most 3 K chunks (each chunk's partial
    costs a write and a serial read in the reduction: 16 chunks measured up
    to 7x slower than 1)."""
    for m_max, lay, s in SK_TABLE.get((N, K), ()):
        if M <= m_max and N % SK_LAYOUTS[lay][0] == 0:
            return lay, s
    KT = K // 64
    best, best_t = (7, 1), float("inf")
    for lay in layouts:
        bn, bm, occ, eff = SK_LAYOUTS[lay]
        if N % bn:
            continue
        tiles = -(-M // bm) * (N // bn)
        for s in (1, 2, 3):
            if s > KT or (s > 1 and KT // s < 8) or (epi == "swiglu" and s > 1):
                continue
            grid = tiles * s
            rounds = -(-grid // (SK_CUS * occ))
            t = rounds * occ * bm * bn * (KT / s) / eff + (s - 1) * bm * bn * 64.0
            if t < best_t:
                best, best_t = (lay, s), t
    return best


_SK_WS_GRAPHS: list = []   # workspaces owned by captured graphs (never reused)


def _sk_workspace(dev: torch.device, stream: int, floats: int, tiles: int):
    """Split-K partials + arrival counters (zero on entry; each tile's reducer
    re-zeroes its own). Eager launches share one growing workspace per stream
    (stream order serialises them). A launch being CAPTURED gets a workspace of
    its own that lives as long as the process: a shared one could be regrown
    by a later capture, freeing memory an earlier graph still replays into,
    and two graphs replayed on different streams would race on it."""
    if dev.type == "cuda" and torch.cuda.is_current_stream_capturing():
        ws = (torch.empty(floats, dtype=torch.float32, device=dev),
              torch.zeros(tiles, dtype=torch.int32, device=dev))
        _SK_WS_GRAPHS.append(ws)
        return ws
    key = (dev, stream)
    ws = _SK_WS.get(key)
    if ws is None or ws[0].numel() < floats or ws[1].numel() < tiles:
        f = max(floats, 0 if ws is None else ws[0].numel())
        t = max(tiles, 0 if ws is None else ws[1].numel())
        ws = (torch.empty(f, dtype=torch.float32, device=dev),
              torch.zeros(t, dtype=torch.int32, device=dev))
        _SK_WS[key] = ws
    return ws


def _sk_ref(x: torch.Tensor, w: torch.Tensor, epi: str, bias, residual, act: str | None = None):
    y = x.float() @ w.float().t()
    if epi == "swiglu":
        F = w.shape[0] // 2
        g = y[:, :F].to(torch.bfloat16).float()
        u = y[:, F:].to(torch.bfloat16).float()
        return (g * torch.sigmoid(g) * u).to(torch.bfloat16)
    if bias is not None:
        y = y + bias.float()
    if epi == "resid":
        return (residual.float() + y).to(torch.bfloat16)
    if act == "gelu":
        y = y.to(torch.bfloat16).float()
        y = 0.5 * y * (1.0 + torch.erf(y * 0.70710678118654752))
    return y.to(torch.bfloat16)


def gemm_sk(x: torch.Tensor, w: torch.Tensor, *, epi: str = "bf16", bias: torch.Tensor | None = None,
            act: str | None = None, residual: torch.Tensor | None = None,
            out: torch.Tensor | None = None, layout: int | None = None,
            splits: int | None = None) -> torch.Tensor:
    """Y = X W^T on the split-K tiled GEMM (``csrc/kernels/gemm_sk.hip``); the
    S K-chunks of a tile are summed in-launch by the tile's last workgroup.

    x [M, K] bf16 (row stride may exceed K), w [N, K] bf16 row-major.
    ``epi``: "bf16" -> [M, N] (+ f32 ``bias``, ``act`` "gelu"); "swiglu" -> silu(gate) * up
    [M, N / 2] (gate rows [0, N/2), up rows [N/2, N)); "resid" -> ``residual``
    [M, N] += X W^T (+ ``bias``) in place (one bf16 rounding), returned."""
    N, K = w.shape
    M = x.shape[0]
    assert x.shape[1] == K, (x.shape, w.shape)
    if epi == "resid":
        assert residual is not None and residual.shape == (M, N)
    if not _gpu(x):
        y = _sk_ref(x, w, epi, bias, residual, act)
        dst = residual if epi == "resid" else out
        if dst is not None:
            dst.copy_(y)
            return dst
        return y
    if x.dtype != torch.bfloat16 or w.dtype != torch.bfloat16:
        raise TypeError("gemm_sk needs bf16 operands")
    if x.stride(1) != 1 or not w.is_contiguous():
        raise ValueError("gemm_sk needs K-contiguous operands")
    if layout is None or splits is None:
        pl, ps = gemm_sk_plan(M, N, K, epi)
        layout = pl if layout is None else layout
        splits = ps if splits is None else splits
    bn, bm = SK_LAYOUTS[layout][:2]
    if N % bn or K % 64:
        raise ValueError(f"gemm_sk layout {layout}: N {N} / K {K} not tileable")
    p = _lib.GemmSkParams()
    p.x, p.ldx, p.w = ptr(x), x.stride(0), ptr(w)
    p.M, p.N, p.K, p.S, p.epi = M, N, K, splits, _SK_EPI[epi]
    p.act = 1 if act == "gelu" else 0
    assert not act or epi == "bf16"
    if bias is not None:
        assert epi != "swiglu" and bias.dtype == torch.float32 and bias.is_contiguous() and bias.numel() == N
    p.bias = ptr(bias)
    if epi == "resid":
        y = residual
        assert y.dtype == torch.bfloat16 and y.stride(1) == 1
    else:
        cols = N // 2 if epi == "swiglu" else N
        y = out if out is not None else torch.empty(M, cols, dtype=torch.bfloat16, device=x.device)
        assert y.shape == (M, cols) and y.stride(1) == 1
    p.y, p.ldy = ptr(y), y.stride(0)
    st = stream_ptr(x)
    if splits > 1:
        tiles = -(-M // bm) * (N // bn)
        ws, cnt = _sk_workspace(x.device, st, tiles * splits * bm * bn, tiles)
        p.ws, p.counters = ptr(ws), ptr(cnt)
    p.layout = layout
    check(kernels().loqa_gemm_sk(ctypes.byref(p), st), "gemm_sk")
    return y


# ---------------------------------------------------------------------------
# Row-resident weight-streaming GEMM (csrc/kernels/gemm_ws.hip)
_WS_EPI = {"bf16": 0, "swiglu": 1, "resid": 2}
WS_MAX_BM = 384


def gemm_ws_rows(M: int, depth: int = 0) -> int:
    """Rows per workgroup: M split into the fewest blocks of <= 384 rows
    (<= 256 at depth 1), each rounded up to 64."""
    cap = WS_MAX_BM if depth == 0 else 256
    nb = -(-M // cap)
    return -(-(-(-M // nb)) // 64) * 64


def gemm_ws(x: torch.Tensor, w: torch.Tensor, *, epi: str = "bf16", bias: torch.Tensor | None = None,
            act: str | None = None, residual: torch.Tensor | None = None,
            out: torch.Tensor | None = None, depth: int | None = None,
            bm: int | None = None, splits: int = 1) -> torch.Tensor:
    """Y = X W^T on the row-resident weight-streaming GEMM: a workgroup owns
    128 output features x all the rows of its row block (up to 384), so every
    weight byte is read once; ``splits`` K chunks per tile, summed in-launch.
    Epilogues as :func:`gemm_sk`."""
    N, K = w.shape
    M = x.shape[0]
    assert x.shape[1] == K, (x.shape, w.shape)
    if epi == "resid":
        assert residual is not None and residual.shape == (M, N)
    if not _gpu(x):
        y = _sk_ref(x, w, epi, bias, residual, act)
        dst = residual if epi == "resid" else out
        if dst is not None:
            dst.copy_(y)
            return dst
        return y
    if x.dtype != torch.bfloat16 or w.dtype != torch.bfloat16:
        raise TypeError("gemm_ws needs bf16 operands")
    if x.stride(1) != 1 or not w.is_contiguous() or N % 128 or K % 64:
        raise ValueError("gemm_ws needs K-contiguous operands, N % 128 == 0, K % 64 == 0")
    depth = 0 if depth is None else depth
    p = _lib.GemmWsParams()
    p.x, p.ldx, p.w = ptr(x), x.stride(0), ptr(w)
    p.M, p.N, p.K, p.epi = M, N, K, _WS_EPI[epi]
    p.act = 1 if act == "gelu" else 0
    assert not act or epi == "bf16"
    if bias is not None:
        assert epi != "swiglu" and bias.dtype == torch.float32 and bias.is_contiguous() and bias.numel() == N
    p.bias = ptr(bias)
    if epi == "resid":
        y = residual
        assert y.dtype == torch.bfloat16 and y.stride(1) == 1
    else:
        cols = N // 2 if epi == "swiglu" else N
        y = out if out is not None else torch.empty(M, cols, dtype=torch.bfloat16, device=x.device)
        assert y.shape == (M, cols) and y.stride(1) == 1
    p.y, p.ldy = ptr(y), y.stride(0)
    p.bm = gemm_ws_rows(M, depth) if bm is None else bm
    p.S = splits
    st = stream_ptr(x)
    if splits > 1:
        tiles = -(-M // p.bm) * (N // 128)
        ws, cnt = _sk_workspace(x.device, st, tiles * splits * p.bm * 128, tiles)
        p.ws, p.counters = ptr(ws), ptr(cnt)
    check(kernels().loqa_gemm_ws(ctypes.byref(p), depth, st), "gemm_ws")
    return y


# ---------------------------------------------------------------------------
# Projection dispatch for prompt passes (prefill, Whisper encoder): the
# hand-written GEMM measured fastest per (N, K) and row count
# (scripts/exp/gemm_sk_bench.py --grid, cold weights; profiles/r4_gemm_proj_grid.txt):
# ("sk", layout, K chunks) = gemm_sk, ("ws", depth[, K chunks]) = gemm_ws.
PROJ_TABLE = {
    # the chunked prompt passes (LOQA_CHUNK_PREFILL) also run 64-256 rows:
    # more K chunks fill the CUs there (profiles/r4_gemm_small_m.txt; a 32 /
    # 128-row pass 4.81 / 6.33 vs 6.70 / 7.21 ms, headline neutral:
    # profiles/r4_ab_proj_small_m.txt)
    (6144, 4096): [(64, ("sk", 4, 4)), (128, ("sk", 4, 2)), (400, ("sk", 4, 1)),
                   (900, ("sk", 5, 1)), (1 << 30, ("sk", 0, 1))],                         # Llama qkv
    (4096, 4096): [(128, ("sk", 4, 4)), (256, ("sk", 4, 2)), (900, ("sk", 4, 1)),
                   (1 << 30, ("sk", 0, 1))],                                               # o
    (28672, 4096): [(256, ("ws", 1)), (384, ("ws", 0)), (900, ("ws", 0)),
                    (1 << 30, ("sk", 6, 1))],                                              # gate|up
    # 400-1000 rows (whole-prompt passes of two or three prompts, nothing
    # decoding): down on the weight-streaming GEMM with K chunks, gate|up on it
    # unsplit (600 rows: 94 vs 118 us, 160 vs 196 us; profiles/r4_ws_splitk.txt).
    # At 300-400 rows, the chunked passes beside the Whisper decoder, the split-K
    # weight-streaming down too: round 4's 3 pairs read neutral (19.03 vs 19.07),
    # round 5's 5 interleaved pairs all favour it - mixed pass 13.0 -> 12.4 ms,
    # +1.2% utt/s (profiles/r5_ab_down_ws.txt)
    (4096, 14336): [(64, ("sk", 4, 8)), (128, ("sk", 5, 8)), (256, ("sk", 5, 4)),
                    (400, ("ws", 0, 4)), (700, ("ws", 0, 4)), (1000, ("ws", 0, 2)),
                    (1 << 30, ("sk", 6, 3))],                                              # down
    # encoder qkv / fc1: gemm_ws is ~8% faster alone (24.2 / 25.8 vs 26.2 / 28.2
    # us) but its long-lived 512-thread workgroups cost the concurrent decoders
    # more than that (encoder on ws: 18.82 / 19.02 vs 19.15 / 18.99 utt/s)
    (3840, 1280): [(2000, ("sk", 1, 1)), (1 << 30, ("sk", 6, 1))],                        # enc qkv
    (1280, 1280): [(2000, ("sk", 4, 1)), (1 << 30, ("sk", 5, 1))],                        # enc o
    (5120, 1280): [(2000, ("sk", 0, 1)), (1 << 30, ("sk", 6, 1))],                        # enc fc1
    (1280, 5120): [(2000, ("sk", 4, 1)), (1 << 30, ("sk", 5, 1))],                        # enc fc2
    # Llama-3-70B TP=8 shards, prompt passes of ~320 rows (grid search,
    # profiles/r5_tp70_shard_grid.jsonl): the planner's (4, 2) / (5, 1) picks
    # were 38.1 / 85.3 us, these 27.2 / 69.7 us (hipBLASLt 28.1 / 69.8); o and
    # down shards keep the planner's (5, 1) (15.2 / 37.6 us)
    # deeper LDS rings (layouts 9 / 11, profiles/r5_sk_grid_deep.jsonl): 25.6 /
    # 62.9 us vs 26.9 / 68.9 (a TP rank runs no decoder beside its prompt pass)
    (1280, 8192): [(512, ("sk", 11, 4))],                                                  # qkv/8
    (7168, 8192): [(512, ("sk", 9, 3))],                                                   # gate|up/8
}
# the 8B prompt-pass projections at ~300 rows on the 4-stage rings (qkv 32.7 ->
# 30.3, o 32.0 -> 30.2, down 76.3 -> 73.4 us alone; one workgroup per CU
# instead of two beside the decoders): LOQA_SK_DEEP
SK_DEEP = os.environ.get("LOQA_SK_DEEP", "0") == "1"
# experiment override of the <= 400-row (chunked prompt pass) pick of a shape:
# "NxK:sk,layout,chunks;NxK:ws,depth,chunks"
for _ov in filter(None, os.environ.get("LOQA_PROJ_OVERRIDE", "").split(";")):
    try:
        _shape, _pick = _ov.split(":")
        _n, _k = map(int, _shape.split("x"))
        _kind, *_args = _pick.split(",")
        if _kind not in ("sk", "ws"):
            raise ValueError(_kind)
        PROJ_TABLE[(_n, _k)] = [(400, (_kind, *map(int, _args)))] + [
            e for e in PROJ_TABLE.get((_n, _k), []) if e[0] > 400]
    except ValueError:
        import warnings
        warnings.warn(f"LOQA_PROJ_OVERRIDE: ignoring malformed entry {_ov!r}")
if SK_DEEP:
    PROJ_TABLE[(6144, 4096)].insert(2, (400, ("sk", 11, 1)))
    PROJ_TABLE[(4096, 4096)].insert(2, (400, ("sk", 11, 1)))
    PROJ_TABLE[(4096, 14336)][3] = (400, ("sk", 9, 4))


def proj(x: torch.Tensor, w: torch.Tensor, *, epi: str = "bf16", bias: torch.Tensor | None = None,
         act: str | None = None, residual: torch.Tensor | None = None) -> torch.Tensor:
    """A prompt-pass projection on the fastest hand-written GEMM for its shape
    (``PROJ_TABLE``; shapes outside it: the gemm_sk planner). Epilogues as
    :func:`gemm_sk`."""
    M = x.shape[0]
    N, K = w.shape
    choice = None
    for m_max, c in PROJ_TABLE.get((N, K), ()):
        if M <= m_max:
            choice = c
            break
    if choice is not None and choice[0] == "ws" and N % 128 == 0:
        return gemm_ws(x, w, epi=epi, bias=bias, act=act, residual=residual, depth=choice[1],
                       splits=choice[2] if len(choice) > 2 else 1)
    if choice is not None and choice[0] == "sk" and N % SK_LAYOUTS[choice[1]][0] == 0:
        return gemm_sk(x, w, epi=epi, bias=bias, act=act, residual=residual, layout=choice[1],
                       splits=choice[2])
    return gemm_sk(x, w, epi=epi, bias=bias, act=act, residual=residual)
