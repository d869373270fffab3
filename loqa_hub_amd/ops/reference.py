"""Plain-PyTorch fp32 reference implementations of every hot op.

These are the numerics oracle for the HIP kernels (tests compare kernel output
against them) and the CPU execution path (no GPU in the CI tier).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import torch


def rmsnorm(x, w, eps, residual=None):
    if residual is not None:
        s = (x.float() + residual.float()).to(residual.dtype)
        residual.copy_(s)
        x = s
    xf = x.float()
    y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * w.float()
    return y.to(x.dtype)


def layernorm(x, w, b, eps, residual=None):
    if residual is not None:
        s = (x.float() + residual.float()).to(residual.dtype)
        residual.copy_(s)
        x = s
    y = torch.nn.functional.layer_norm(x.float(), (x.shape[-1],), w.float(), b.float(), eps)
    return y.to(x.dtype)


def silu_mul(x):
    F = x.shape[-1] // 2
    g, u = x[..., :F].float(), x[..., F:].float()
    return (torch.nn.functional.silu(g) * u).to(x.dtype)


def gelu_bias_(x, bias=None, pos=None):
    y = x.float()
    if bias is not None:
        y = y + bias.float()
    y = torch.nn.functional.gelu(y)
    if pos is not None:
        rows = y.reshape(-1, y.shape[-1]).shape[0]
        idx = torch.arange(rows, device=x.device) % pos.shape[0]
        y = (y.reshape(-1, y.shape[-1]) + pos.float()[idx]).reshape(y.shape)
    x.copy_(y.to(x.dtype))
    return x


def rope_cos_sin(head_dim: int, max_pos: int, theta: float, device=None,
                 scaling: tuple | None = None) -> torch.Tensor:
    """[max_pos, D/2, 2] f32 table of (cos, sin) for NeoX rotate-half RoPE.
    ``scaling`` = (factor, low_freq_factor, high_freq_factor, original max
    positions): Llama-3.1 frequency scaling - wavelengths longer than
    original / low are divided by ``factor``, shorter than original / high
    kept, and the band between interpolated."""
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    if scaling is not None:
        factor, low, high, orig = scaling
        wavelen = 2 * math.pi / inv
        smooth = ((orig / wavelen - low) / (high - low)).clamp(0.0, 1.0)
        inv = torch.where(wavelen > orig / low, inv / factor,
                          torch.where(wavelen < orig / high, inv,
                                      (1 - smooth) * inv / factor + smooth * inv))
    ang = torch.arange(max_pos, dtype=torch.float64)[:, None] * inv[None, :]
    return torch.stack([ang.cos(), ang.sin()], dim=-1).float().to(device)


def apply_rope(x: torch.Tensor, cs: torch.Tensor) -> torch.Tensor:
    """x [T, H, D] (any float), cs [T, D/2, 2] -> rotated x (fp32)."""
    half = x.shape[-1] // 2
    a, b = x[..., :half].float(), x[..., half:].float()
    c, s = cs[:, None, :, 0], cs[:, None, :, 1]
    return torch.cat([a * c - b * s, b * c + a * s], dim=-1)


def rope_kv_append(qkv, positions, cos_sin, k_cache, v_cache, slots, H, Hkv, D):
    T = qkv.shape[0]
    if T == 0:
        return None
    q = qkv[:, : H * D].view(T, H, D)
    k = qkv[:, H * D:(H + Hkv) * D].view(T, Hkv, D)
    v = qkv[:, (H + Hkv) * D:(H + 2 * Hkv) * D].view(T, Hkv, D)
    if cos_sin is not None:
        cs = cos_sin[positions.long()]
        q.copy_(apply_rope(q, cs).to(q.dtype))
        k = apply_rope(k, cs).to(qkv.dtype)
    blk = k_cache.shape[2]
    sl = slots.long()
    valid = sl >= 0
    b, o = (sl // blk)[valid], (sl % blk)[valid]
    k_cache[b, :, o, :] = k[valid].to(k_cache.dtype)
    v_cache[b, :, o, :] = v[valid].to(v_cache.dtype)
    return None


def attention(q, k, v, cu_q, *, n_heads, n_kv, head_dim, causal, cu_k=None, ctx_lens=None,
              block_tables=None, scale=None, out=None):
    H, Hkv, D = n_heads, n_kv, head_dim
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    Tq = q.shape[0]
    res = torch.zeros(Tq, H * D, dtype=torch.float32, device=q.device)
    cuq = cu_q.tolist()
    G = H // Hkv
    for b in range(len(cuq) - 1):
        q0, q1 = cuq[b], cuq[b + 1]
        ql = q1 - q0
        if ql == 0:
            continue
        if block_tables is not None:
            L = int(ctx_lens[b])
            blk = k.shape[2]
            idx = torch.arange(L, device=k.device)
            bt = block_tables[b].long()[idx // blk]
            kb = k[bt, :, idx % blk, :].float()  # [L, Hkv, D]
            vb = v[bt, :, idx % blk, :].float()
        else:
            k0 = int(cu_k[b])
            k1 = k0 + int(ctx_lens[b]) if ctx_lens is not None else int(cu_k[b + 1])
            L = k1 - k0
            kb = k[k0:k1, : Hkv * D].reshape(L, Hkv, D).float()
            vb = v[k0:k1, : Hkv * D].reshape(L, Hkv, D).float()
        qb = q[q0:q1, : H * D].reshape(ql, H, D).float()
        kb = kb.repeat_interleave(G, dim=1)
        vb = vb.repeat_interleave(G, dim=1)
        s = torch.einsum("qhd,khd->hqk", qb, kb) * scale
        if causal:
            qpos = torch.arange(ql, device=q.device) + (L - ql)
            kpos = torch.arange(L, device=q.device)
            s = s.masked_fill(kpos[None, None, :] > qpos[None, :, None], float("-inf"))
        p = torch.softmax(s, dim=-1)
        p = torch.nan_to_num(p, nan=0.0)
        res[q0:q1] = torch.einsum("hqk,khd->qhd", p, vb).reshape(ql, H * D)
    r = res.to(q.dtype)
    if out is not None:
        out.copy_(r)
        return out
    return r


def masked_argmax(logits, mask=None, mask_rows=None):
    x = logits.float()
    B, V = x.shape
    if mask is not None:
        m = mask if mask_rows is None else mask[mask_rows.long()]
        bits = unpack_mask(m, V)
        x = x.masked_fill(~bits, float("-inf"))
        none = ~bits.any(dim=-1)
    else:
        none = torch.zeros(B, dtype=torch.bool, device=x.device)
    r = x.argmax(dim=-1).to(torch.int32)
    r[none] = -1
    return r


def unpack_mask(m: torch.Tensor, V: int) -> torch.Tensor:
    """int32 words [..., W] -> bool [..., V]"""
    shifts = torch.arange(32, device=m.device, dtype=torch.int32)
    bits = (m.unsqueeze(-1) >> shifts) & 1
    return bits.reshape(*m.shape[:-1], -1)[..., :V].bool()


def pack_mask(bits: torch.Tensor) -> torch.Tensor:
    """bool [..., V] -> int32 words [..., ceil(V/32)]"""
    V = bits.shape[-1]
    W = (V + 31) // 32
    pad = torch.zeros(*bits.shape[:-1], W * 32, dtype=torch.int64, device=bits.device)
    pad[..., :V] = bits.long()
    w = (pad.reshape(*bits.shape[:-1], W, 32) << torch.arange(32, device=bits.device)).sum(-1)
    w = torch.where(w >= 2**31, w - 2**32, w)
    return w.to(torch.int32)


def pcm16_to_f32_sumsq(pcm, offsets):
    f = pcm.float() / 32767.0
    off = offsets.tolist()
    ss = torch.tensor([float((f[off[i]:off[i + 1]].double() ** 2).sum()) for i in range(len(off) - 1)],
                      dtype=torch.float32)
    return f, ss


# ------------------------------------------------------------- log-mel consts
def _hz_to_mel(f):
    f = np.asarray(f, dtype=np.float64)
    f_sp = 200.0 / 3
    mels = f / f_sp
    min_log_hz = 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = np.log(6.4) / 27.0
    return np.where(f >= min_log_hz, min_log_mel + np.log(np.maximum(f, 1e-10) / min_log_hz) / logstep, mels)


def _mel_to_hz(m):
    m = np.asarray(m, dtype=np.float64)
    f_sp = 200.0 / 3
    freqs = f_sp * m
    min_log_hz = 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = np.log(6.4) / 27.0
    return np.where(m >= min_log_mel, min_log_hz * np.exp(logstep * (m - min_log_mel)), freqs)


def mel_filterbank(sr: int = 16000, n_fft: int = 400, n_mels: int = 80) -> np.ndarray:
    """Slaney-style mel filterbank (librosa defaults, as whisper uses)."""
    n_freqs = 1 + n_fft // 2
    fftfreqs = np.linspace(0, sr / 2, n_freqs)
    mel_f = _mel_to_hz(np.linspace(_hz_to_mel(0.0), _hz_to_mel(sr / 2), n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = mel_f[:, None] - fftfreqs[None, :]
    lower = -ramps[:-2] / fdiff[:-1, None]
    upper = ramps[2:] / fdiff[1:, None]
    w = np.maximum(0, np.minimum(lower, upper))
    enorm = 2.0 / (mel_f[2: n_mels + 2] - mel_f[:n_mels])
    return (w * enorm[:, None]).astype(np.float32)


@dataclass
class MelConstants:
    n_mels: int
    window: torch.Tensor      # [400]
    cos_basis: torch.Tensor   # [400, 224]
    sin_basis: torch.Tensor   # [400, 224]
    filters: torch.Tensor     # [n_mels, 201]

    @staticmethod
    def create(n_mels: int = 80) -> "MelConstants":
        n = np.arange(400)
        window = (0.5 - 0.5 * np.cos(2 * np.pi * n / 400)).astype(np.float32)  # periodic Hann
        k = np.arange(224)
        ang = 2 * np.pi * np.outer(n, k) / 400
        cosb = np.cos(ang)
        sinb = -np.sin(ang)
        cosb[:, 201:] = 0
        sinb[:, 201:] = 0
        return MelConstants(n_mels, torch.from_numpy(window), torch.from_numpy(cosb.astype(np.float32)),
                            torch.from_numpy(sinb.astype(np.float32)),
                            torch.from_numpy(mel_filterbank(n_mels=n_mels)))

    def to(self, device) -> "MelConstants":
        device = torch.device(device)
        if self.window.device == device:
            return self
        cache = self.__dict__.setdefault("_dev_cache", {})
        key = str(device)
        if key not in cache:
            cache[key] = MelConstants(self.n_mels, self.window.to(device), self.cos_basis.to(device),
                                      self.sin_basis.to(device), self.filters.to(device))
        return cache[key]


def log_mel(audio: torch.Tensor, c: MelConstants) -> torch.Tensor:
    """Whisper log-mel (whisper/audio.py semantics) in fp32: [B, n_mels, n//160]."""
    win = c.window.to(audio.device)
    st = torch.stft(audio.float(), 400, 160, window=win, return_complex=True, center=True,
                    pad_mode="reflect")
    mag = st[..., :-1].abs() ** 2
    mel = c.filters.to(audio.device) @ mag
    lg = torch.clamp(mel, min=1e-10).log10()
    mx = lg.amax(dim=(-2, -1), keepdim=True)
    lg = torch.maximum(lg, mx - 8.0)
    return (lg + 4.0) / 4.0


def im2col_k3(x, strides, B, C, L, stride):
    Lout = (L - 1) // stride + 1
    flat = x.reshape(-1)
    b = torch.arange(B, device=x.device)[:, None, None, None]
    to = torch.arange(Lout, device=x.device)[None, :, None, None]
    c = torch.arange(C, device=x.device)[None, None, :, None]
    k = torch.arange(3, device=x.device)[None, None, None, :]
    t = to * stride + k - 1
    valid = (t >= 0) & (t < L)
    idx = b * strides[0] + c * strides[1] + t.clamp(0, L - 1) * strides[2]
    vals = flat[idx.reshape(-1)].reshape(B, Lout, C, 3)
    vals = torch.where(valid.expand(B, Lout, C, 3), vals, torch.zeros((), dtype=x.dtype))
    return vals.reshape(B * Lout, 3 * C)


# ----------------------------------------------------------- decode slabs
def shuffle_weight(w):
    N, K = w.shape
    return w.reshape(N // 16, 16, K // 32, 4, 8).permute(0, 2, 3, 1, 4).contiguous().reshape(
        N // 16, K // 32, 64, 8)


def unshuffle_weight(wp):
    T, KS = wp.shape[:2]
    return wp.reshape(T, KS, 4, 16, 8).permute(0, 3, 1, 2, 4).reshape(T * 16, KS * 32)


def skinny_gemm(x, wp, S):
    w = unshuffle_weight(wp)
    Mpad, K = x.shape
    kc = K // S
    parts = [x[:, s * kc:(s + 1) * kc].float() @ w[:, s * kc:(s + 1) * kc].float().t() for s in range(S)]
    return torch.stack(parts, 0)


def slab_rmsnorm(part, residual, w, eps, row_idx=None, write_residual=True):
    tot = part.sum(0)
    idx = row_idx.long() if row_idx is not None else torch.arange(part.shape[1], device=part.device)
    s = (tot[idx] + residual[idx].float()).to(residual.dtype)
    if write_residual:
        residual[idx] = s
    xf = s.float()
    y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * w.float()
    return y.to(residual.dtype)


def slab_rope_append(part, positions, cos_sin, k_cache, v_cache, slots, H, Hkv, D, bias=None):
    tot = part.sum(0)
    if bias is not None:
        tot = tot + bias.float()
    qkv = tot.to(torch.bfloat16)
    rope_kv_append(qkv, positions, cos_sin, k_cache, v_cache, slots, H, Hkv, D)
    return qkv[:, : H * D].contiguous()


def slab_layernorm(part, residual, w, b, eps, bias=None, row_idx=None, write_residual=True):
    tot = part.sum(0)
    if bias is not None:
        tot = tot + bias.float()
    tot = tot.to(torch.bfloat16).float()
    idx = row_idx.long() if row_idx is not None else torch.arange(part.shape[1], device=part.device)
    s = (tot[idx] + residual[idx].float()).to(residual.dtype)
    if write_residual:
        residual[idx] = s
    return torch.nn.functional.layer_norm(s.float(), (s.shape[-1],), w.float(), b.float(),
                                          eps).to(residual.dtype)


def slab_bias_act(part, bias=None, act="none"):
    tot = part.sum(0)
    if bias is not None:
        tot = tot + bias.float()
    if act == "gelu":
        tot = torch.nn.functional.gelu(tot.to(torch.bfloat16).float())
    return tot.to(torch.bfloat16)


def slab_silu_mul(part):
    return silu_mul(part.sum(0).to(torch.bfloat16))


# ------------------------------------------------------------------ VITS / HiFi-GAN
def conv1d(x, w, bias=None, *, dil=1, pad=0, stride=1, pre_slope=None, act=None, res=None,
           alpha=1.0, acc=None, lens=None, Tout=None, ostride=1, ophase=0, Tq=None):
    """Reference of loqa_conv1d: x [B, Tin, Cin] (channels-last), w [Cout, Cin, K]
    (torch layout) -> y [B, Tout, Cout'] following the kernel's epilogue order.
    Returns float32 (callers round)."""
    B, Tin, Cin = x.shape
    xf = x.float()
    if pre_slope is not None:
        xf = torch.nn.functional.leaky_relu(xf, pre_slope)
    xf = xf.to(torch.bfloat16).float()  # the kernel feeds bf16 operands to the MFMA
    y = torch.nn.functional.conv1d(xf.transpose(1, 2), w.float(), None, stride=stride, padding=pad,
                                   dilation=dil).transpose(1, 2)
    if Tq is not None:
        y = y[:, :Tq]
    if bias is not None:
        y = y + bias.float()
    if act == "relu":
        y = torch.relu(y)
    elif act == "tanh":
        y = torch.tanh(y)
    elif act == "gated":
        Hh = y.shape[-1] // 2
        a, g = y[..., :Hh].to(torch.bfloat16).float(), y[..., Hh:].to(torch.bfloat16).float()
        y = torch.tanh(a) * torch.sigmoid(g)
    T_out = Tout if Tout is not None else y.shape[1] * ostride + ophase
    full = torch.zeros(B, T_out, y.shape[-1], dtype=torch.float32, device=x.device)
    q = torch.arange(y.shape[1], device=x.device)
    oi = q * ostride + ophase
    ok = (oi >= 0) & (oi < T_out)
    full[:, oi[ok]] = y[:, q[ok]]
    idx = oi[ok]
    if res is not None:
        full[:, idx] += res[:, idx].float()
    full[:, idx] *= alpha
    if acc is not None:
        full[:, idx] += acc[:, idx].float()
    if lens is not None:
        t = torch.arange(T_out, device=x.device)
        full = full * (t[None, :] < lens[:, None].to(x.device)).float()[..., None]
    return full


def conv_transpose1d(x, w, bias=None, *, stride, padding, pre_slope=None):
    """torch ConvTranspose1d on channels-last x; w [Cin, Cout, K] torch layout."""
    xf = x.float()
    if pre_slope is not None:
        xf = torch.nn.functional.leaky_relu(xf, pre_slope)
    xf = xf.to(torch.bfloat16).float()
    y = torch.nn.functional.conv_transpose1d(xf.transpose(1, 2), w.float(),
                                             None if bias is None else bias.float(),
                                             stride=stride, padding=padding)
    return y.transpose(1, 2)


def relpos_attention(qkv, emb_k, emb_v, lens, H, D, window, scale):
    B, T, _ = qkv.shape
    C = H * D
    q = qkv[..., :C].float().view(B, T, H, D).transpose(1, 2) * scale
    k = qkv[..., C:2 * C].float().view(B, T, H, D).transpose(1, 2)
    v = qkv[..., 2 * C:3 * C].float().view(B, T, H, D).transpose(1, 2)
    s = q @ k.transpose(-1, -2)
    idx = torch.arange(T, device=qkv.device)
    rel = idx[None, :] - idx[:, None]
    inwin = rel.abs() <= window
    ek = emb_k.float()
    rl = torch.einsum("bhid,rd->bhir", q, ek)  # [B,H,T,2w+1]
    ridx = (rel + window).clamp(0, 2 * window)
    s = s + torch.where(inwin, rl.gather(-1, ridx[None, None].expand(B, H, T, T)),
                        torch.zeros((), device=qkv.device))
    L = lens.to(qkv.device) if lens is not None else torch.full((B,), T, device=qkv.device)
    valid = idx[None, :] < L[:, None]
    m = valid[:, None, :, None] & valid[:, None, None, :]
    s = s.masked_fill(~m, -1e4)
    p = torch.softmax(s, -1)
    o = p @ v
    pw = torch.where(inwin, p, torch.zeros((), device=qkv.device))
    pr = torch.zeros(B, H, T, 2 * window + 1, device=qkv.device)
    pr.scatter_add_(-1, ridx[None, None].expand(B, H, T, T), pw)
    o = o + pr @ emb_v.float()
    o = o * valid[:, None, :, None]
    return o.transpose(1, 2).reshape(B, T, C)


def expand_sample(stats, cum, flen, F, noise_scale, noise=None):
    """z[b, f] = m[i(f)] + noise * exp(logs[i(f)]) * noise_scale."""
    B, T, C2 = stats.shape
    C = C2 // 2
    z = torch.zeros(B, F, C, device=stats.device)
    for b in range(B):
        n = int(flen[b])
        f = torch.arange(n, device=stats.device)
        i = torch.searchsorted(cum[b].to(stats.device), f, right=True)
        m, lg = stats[b, i, :C].float(), stats[b, i, C:].float()
        e = noise[b, :n].float() if noise is not None else torch.zeros_like(m)
        z[b, :n] = m + e * torch.exp(lg) * noise_scale
    return z


# ------------------------------------------------------------ fused decode GEMMs
def perm_rope_qkv(H, Hkv, D):
    """Row order of the fused qkv weight: per q / k head, 16-row pair tiles
    holding 8 first-half rows c0.. and their RoPE partners c0 + D/2 (the
    epilogue pairs lane l with lane l ^ 32); v rows unchanged."""
    half = D // 2
    rows = []
    for base, n in ((0, H), (H * D, Hkv)):
        for h in range(n):
            for s in range(D // 16):
                c0 = 8 * s
                rows += list(range(base + h * D + c0, base + h * D + c0 + 8))
                rows += list(range(base + h * D + half + c0, base + h * D + half + c0 + 8))
    rows += list(range((H + Hkv) * D, (H + 2 * Hkv) * D))
    return torch.tensor(rows, dtype=torch.long)


def perm_gate_up(F):
    """Row order of the fused gate|up weight: 16-row pair tiles of (8 gate, 8 up)."""
    rows = []
    for t in range(F // 8):
        rows += list(range(8 * t, 8 * t + 8)) + list(range(F + 8 * t, F + 8 * t + 8))
    return torch.tensor(rows, dtype=torch.long)


def swiglu_pairs(y):
    """silu(gate) * up of a ``perm_gate_up``-ordered product [M, 2F] (16-column
    pair tiles: 8 gate, 8 up) -> [M, F] (f32)."""
    M, F2 = y.shape
    t = y.float().view(M, F2 // 16, 2, 8)
    g, u = t[:, :, 0], t[:, :, 1]
    g = g.to(torch.bfloat16).float()
    u = u.to(torch.bfloat16).float()
    return (torch.nn.functional.silu(g) * u).reshape(M, F2 // 2)


def fused_ln_stats(rowsq_in, rowsum_in, eps, K):
    """LayerNorm (mean, 1/std) per row from per-tile partial sums [tiles, Mpad]."""
    mean = rowsum_in.float().sum(0) / K
    var = (rowsq_in.float().sum(0) / K - mean * mean).clamp_min(0.0)
    return mean, torch.rsqrt(var + eps)


def fused_row_scale(rowsq_in, eps, K):
    """RMSNorm row scale 1/rms from per-tile partial sums of squares [tiles, Mpad]."""
    tot = rowsq_in.float().sum(0)  # [Mpad]
    return torch.rsqrt(tot / K + eps)


def _fmix32(h: torch.Tensor) -> torch.Tensor:
    m = 0xFFFFFFFF
    h = h ^ (h >> 16)
    h = (h * 0x85EBCA6B) & m
    h = h ^ (h >> 13)
    h = (h * 0xC2B2AE35) & m
    return h ^ (h >> 16)


def init_uniform4(rows: int, cols: int, ld: int, row0: int, col0: int, s: int,
                  scale: float) -> torch.Tensor:
    """CPU twin of elementwise.hip ``init_uniform4_kernel``: bf16 [rows, cols],
    element (r, c) = scale * (sum_k fmix32(4 idx + k + s) / 2^32 - 2) with
    idx = (row0 + r) * ld + col0 + c (uint32 arithmetic, exact f32 sums)."""
    r = torch.arange(rows, dtype=torch.int64)[:, None] + row0
    c = torch.arange(cols, dtype=torch.int64)[None, :] + col0
    idx = (r * ld + c) & 0xFFFFFFFF
    acc = torch.zeros(rows, cols, dtype=torch.float32)
    for k in range(4):
        h = _fmix32((idx * 4 + k + s) & 0xFFFFFFFF)
        acc += (h >> 8).to(torch.float32) * (1.0 / 16777216.0)
    return ((acc - 2.0) * torch.tensor(scale, dtype=torch.float32)).to(torch.bfloat16)


# ------------------------------------------------------------ whole models
def _causal_attn(q, k, v, G: int, scale: float, q0: int = 0):
    """q [T, H, D], k / v [L, Hkv, D] (fp32); query i sits at position q0 + i."""
    k = k.repeat_interleave(G, dim=1)
    v = v.repeat_interleave(G, dim=1)
    s = torch.einsum("qhd,khd->hqk", q, k) * scale
    qpos = torch.arange(q.shape[0], device=q.device) + q0
    kpos = torch.arange(k.shape[0], device=q.device)
    s = s.masked_fill(kpos[None, None, :] > qpos[None, :, None], float("-inf"))
    return torch.einsum("hqk,khd->qhd", torch.softmax(s, dim=-1), v)


@torch.no_grad()
def llama_forward_ref(w, tokens: list[int]) -> torch.Tensor:
    """fp32 forward of a whole Llama model (``LlamaWeights``, unsharded, with
    its row-major layer copies) over one sequence at positions 0..T-1; returns
    fp32 logits [T, V]. Every weight is the model's own bf16 tensor upcast:
    the oracle of the fused bf16 decode path (tests/test_engine_gpu.py)."""
    cfg = w.cfg
    H, Hkv, D, F = w.h, w.hkv, cfg.head_dim, w.f
    dev = w.embed.device
    t = torch.tensor(tokens, dtype=torch.long, device=dev)
    T = t.numel()
    cs = w.cos_sin[:T].float()

    def rms(x, g):
        return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + cfg.norm_eps) * g.float()
    x = w.embed[t].float()
    for L in w.layers:
        h = rms(x, L["attn_norm"])
        qkv = h @ L["wqkv"].float().t()
        q = apply_rope(qkv[:, : H * D].view(T, H, D), cs)
        k = apply_rope(qkv[:, H * D:(H + Hkv) * D].view(T, Hkv, D), cs)
        v = qkv[:, (H + Hkv) * D:].view(T, Hkv, D)
        a = _causal_attn(q, k, v, H // Hkv, 1.0 / math.sqrt(D)).reshape(T, H * D)
        x = x + a @ L["wo"].float().t()
        gu = rms(x, L["mlp_norm"]) @ L["w_gate_up"].float().t()
        x = x + (torch.nn.functional.silu(gu[:, :F]) * gu[:, F:]) @ L["w_down"].float().t()
    return rms(x, w.final_norm) @ w.lm_head.float().t()


@torch.no_grad()
def whisper_decoder_ref(w, tokens: list[int], enc: torch.Tensor) -> torch.Tensor:
    """fp32 Whisper decoder (``WhisperWeights``) over one sequence at positions
    0..T-1 with cross-attention over the encoder states ``enc`` [T_enc, d];
    returns fp32 logits [T, vocab] (tied embedding)."""
    cfg = w.cfg
    d, H, D = cfg.d_model, cfg.n_heads, cfg.head_dim
    dev = w.tok_embed.device
    t = torch.tensor(tokens, dtype=torch.long, device=dev)
    T = t.numel()
    e = enc.float()

    def ln(x, g, b):
        return torch.nn.functional.layer_norm(x, (d,), g.float(), b.float(), 1e-5)

    def lin(x, W, b):
        return x @ W.float().t() + b.float()

    def gelu(x):
        return 0.5 * x * (1.0 + torch.erf(x * 0.70710678118654752))
    x = w.tok_embed[t].float() + w.dec_pos[:T].float()
    sc = 1.0 / math.sqrt(D)
    for L in w.dec:
        qkv = lin(ln(x, L["ln1_w"], L["ln1_b"]), L["wqkv"], L["bqkv"])
        q, k, v = (qkv[:, i * d:(i + 1) * d].view(T, H, D) for i in range(3))
        x = x + lin(_causal_attn(q, k, v, 1, sc).reshape(T, d), L["wo"], L["bo"])
        q = lin(ln(x, L["lnx_w"], L["lnx_b"]), L["xq"], L["xq_b"]).view(T, H, D)
        kv = lin(e, L["xkv"], L["xkv_b"])
        Te = e.shape[0]
        k, v = kv[:, :d].view(Te, H, D), kv[:, d:].view(Te, H, D)
        p = torch.softmax(torch.einsum("qhd,khd->hqk", q, k) * sc, dim=-1)
        x = x + lin(torch.einsum("hqk,khd->qhd", p, v).reshape(T, d), L["xo"], L["xo_b"])
        x = x + lin(gelu(lin(ln(x, L["ln2_w"], L["ln2_b"]), L["fc1"], L["fc1_b"])), L["fc2"],
                    L["fc2_b"])
    return ln(x, w.dec_ln_w, w.dec_ln_b) @ w.tok_embed.float().t()
