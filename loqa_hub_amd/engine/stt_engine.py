"""Batched on-GPU speech-to-text (Whisper) - replaces the reference's external
OpenAI-compatible STT round trip (``stt_client.go:207-362``: float32->WAV encode,
multipart POST, JSON decode) with: pinned PCM16 -> H2D -> fused convert+RMS
kernel -> log-mel -> encoder -> greedy decoder, batched across utterances.

Random-init weights cannot produce a real transcript, so benchmark/synthetic
requests carry their known transcript and the decoder is *teacher-forced* to it
(SURVEY §7.4 item 1): every step still runs the full decoder forward and the
argmax over the 51 866-entry vocabulary, so cost is that of a real greedy decode
of the same length; only the fed-back token is the reference one.
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field

import numpy as np
import torch

from .. import ops
from ..models.configs import WhisperConfig
from ..models.whisper import WhisperModel, WhisperWeights
from .kv_cache import PagedKVCache
from .tokenizer import get_tokenizer

N_SAMPLES = 480000  # 30 s @ 16 kHz


@dataclass
class STTRequest:
    pcm: np.ndarray                   # int16 samples @ 16 kHz
    transcript: str | None = None     # teacher-forcing target (synthetic mode)
    max_new_tokens: int = 96
    # outputs
    text: str = ""
    sumsq: float = 0.0
    rms: float = 0.0
    tokens: list[int] = field(default_factory=list)
    seq_id: int = -1
    t_done: float = 0.0


class STTEngine:
    def __init__(self, cfg: WhisperConfig, device, *, seed: int = 0, max_batch: int = 64,
                 block_size: int = 16):
        self.cfg = cfg
        self.device = torch.device(device)
        self.weights = WhisperWeights(cfg, self.device, seed=seed)
        self.model = WhisperModel(self.weights)
        self.tok = get_tokenizer(cfg.vocab_size)
        self.sot = [self.tok.token_id(s) for s in
                    ("<|startoftranscript|>", "<|en|>", "<|transcribe|>", "<|notimestamps|>")]
        self.eot = self.tok.token_id("<|endoftext|>")
        self.block_size = block_size
        self.max_blocks = (cfg.n_text_ctx + block_size - 1) // block_size
        self.kv = PagedKVCache(cfg.dec_layers, cfg.n_heads, cfg.head_dim,
                               max_batch * self.max_blocks + 8, block_size, self.device)
        self.is_gpu = self.device.type == "cuda"
        self.ws = ops.AttnWorkspace(self.device, max_batch * 8, cfg.n_heads, cfg.head_dim,
                                    max((cfg.n_audio_ctx + 255) // 256, (cfg.n_text_ctx + 255) // 256)
                                    ) if self.is_gpu else None
        self._next = 1
        self.stats = {"utterances": 0, "decode_steps": 0}

    # ------------------------------------------------------------ front end
    def upload(self, reqs: list[STTRequest], device_pcm: torch.Tensor | None = None
               ) -> tuple[torch.Tensor, torch.Tensor]:
        """PCM16 of all utterances -> one pinned host buffer -> device (side
        stream) -> fused convert + sum-of-squares kernel -> [B, 480000] f32.
        ``device_pcm`` (already on the GPU, e.g. scattered by the DP router
        over RCCL) holds the concatenated samples and skips the H2D copy."""
        lens = [min(len(r.pcm), N_SAMPLES) for r in reqs]
        offs = np.zeros(len(reqs) + 1, np.int64)
        offs[1:] = np.cumsum(lens)
        if device_pcm is not None:
            pcm = device_pcm[: int(offs[-1])]
            off_d = torch.from_numpy(offs).to(self.device)
            f32, sumsq = ops.pcm16_to_f32_sumsq(pcm, off_d)
            return self._pad(f32, offs, lens), sumsq
        host = torch.empty(int(offs[-1]), dtype=torch.int16, pin_memory=self.is_gpu)
        hv = host.numpy()
        for r, o, n in zip(reqs, offs[:-1], lens):
            hv[o:o + n] = r.pcm[:n]
        if self.is_gpu:
            side = torch.cuda.Stream(self.device)
            with torch.cuda.stream(side):
                pcm = host.to(self.device, non_blocking=True)
                off_d = torch.from_numpy(offs).pin_memory().to(self.device, non_blocking=True)
            torch.cuda.current_stream(self.device).wait_stream(side)
            pcm.record_stream(torch.cuda.current_stream(self.device))
            off_d.record_stream(torch.cuda.current_stream(self.device))
        else:
            pcm, off_d = host, torch.from_numpy(offs)
        f32, sumsq = ops.pcm16_to_f32_sumsq(pcm, off_d)
        return self._pad(f32, offs, lens), sumsq

    def _pad(self, f32: torch.Tensor, offs: np.ndarray, lens: list[int]) -> torch.Tensor:
        audio = torch.zeros(len(lens), N_SAMPLES, dtype=torch.float32, device=self.device)
        for i, (o, n) in enumerate(zip(offs[:-1], lens)):
            if n:
                audio[i, :n] = f32[int(o):int(o) + n]
        return audio

    # -------------------------------------------------------------- decode
    def transcribe(self, reqs: list[STTRequest], device_pcm: torch.Tensor | None = None
                   ) -> list[STTRequest]:
        if not reqs:
            return reqs
        audio, sumsq = self.upload(reqs, device_pcm)
        enc = self.model.encode(audio)
        xkv = self.model.cross_kv(enc)
        B = len(reqs)
        T = self.cfg.n_audio_ctx
        targets = []
        for r in reqs:
            r.seq_id = self._next
            self._next += 1
            self.kv.pool.add_seq(r.seq_id, [])
            tgt = None
            if r.transcript is not None:
                tgt = self.tok.encode(" " + r.transcript.strip())[: self.cfg.n_text_ctx - 8] + [self.eot]
            targets.append(tgt)
        feeds = [list(self.sot) for _ in reqs]
        live = list(range(B))
        step = 0
        while live:
            toks, pos, slots, cu, ctx, lidx = [], [], [], [0], [], []
            bt = np.zeros((len(live), self.max_blocks), np.int32)
            max_q, max_ctx = 1, 1
            for j, i in enumerate(live):
                r = reqs[i]
                f = feeds[i]
                start = self.kv.pool.seq_len(r.seq_id)
                sl = self.kv.pool.append(r.seq_id, len(f))
                toks += f
                pos += list(range(start, start + len(f)))
                slots += sl
                cu.append(cu[-1] + len(f))
                ctx.append(start + len(f))
                tab = self.kv.pool.block_table(r.seq_id)
                bt[j, :len(tab)] = tab
                lidx.append(cu[-1] - 1)
                max_q = max(max_q, len(f))
                max_ctx = max(max_ctx, start + len(f))
            dev = lambda a, dt: torch.tensor(a, dtype=dt).to(self.device, non_blocking=True)
            # cross-attention reads each live utterance's 1500 encoder rows in place
            enc_starts = dev([i * T for i in live], torch.int32)
            enc_lens = dev([T] * len(live), torch.int32)
            logits = self.model.decode_step(
                dev(toks, torch.int32), dev(pos, torch.int32), dev(slots, torch.int32),
                dev(cu, torch.int32), dev(ctx, torch.int32), dev(bt, torch.int32), max_q, max_ctx,
                self.kv.k, self.kv.v, xkv, enc_starts, enc_lens, dev(lidx, torch.int64), self.ws)
            nxt = ops.masked_argmax(logits).cpu().numpy()
            self.stats["decode_steps"] += 1
            still = []
            for j, i in enumerate(live):
                r = reqs[i]
                tgt = targets[i]
                t = int(tgt[step]) if tgt is not None else int(nxt[j])
                r.tokens.append(t)
                if t == self.eot or len(r.tokens) >= r.max_new_tokens or (tgt is not None and step + 1 >= len(tgt)):
                    r.t_done = time.perf_counter()
                    continue
                feeds[i] = [t]
                still.append(i)
            live = still
            step += 1
        ss = sumsq.cpu().numpy()
        for i, r in enumerate(reqs):
            n = max(1, min(len(r.pcm), N_SAMPLES))
            r.sumsq = float(ss[i])
            r.rms = float(np.sqrt(ss[i] / n))
            r.text = self.tok.decode([t for t in r.tokens if t != self.eot]).strip()
            self.kv.pool.free_seq(r.seq_id)
        self.stats["utterances"] += B
        return reqs
