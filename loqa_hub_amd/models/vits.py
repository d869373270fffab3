"""VITS text-to-speech (text encoder + duration predictor + reverse flow +
HiFi-GAN generator) on the MI355X path, replacing the reference's external
OpenAI-compatible TTS round trip (``openai_tts_client.go:101-224``).

Layout: every activation is a channels-last bf16 [B, T, C] row tensor, so each
convolution is the MFMA implicit-GEMM kernel of ``conv1d.hip`` with its fused
epilogues:
  text encoder   1x1 QKV conv -> windowed relative-position attention (tts.hip)
                 -> 1x1 out conv (+residual) -> LayerNorm -> FFN (k3 convs,
                 ReLU fused) (+residual) -> LayerNorm, x6; 1x1 projection to
                 (m_p, logs_p)
  durations      deterministic VITS duration predictor (k3 conv + ReLU + LN, x2,
                 1x1 -> log w); random-init weights give arbitrary durations,
                 so they are clamped to [1, 12] frames per symbol
  prior sample   length regulation fused with z_p = m_p + eps exp(logs_p) * 0.667
  flow (reverse) 4 mean-only coupling layers: 1x1 pre conv, WaveNet (k5 conv
                 with the fused gate tanh(a)*sigmoid(b), 1x1 res/skip convs with
                 fused residual / skip accumulation), 1x1 post conv fused with
                 x1 <- x1 - m, channel flip
  decoder        conv_pre k7 -> [leaky-ReLU + ConvTranspose1d (polyphase MFMA)
                 -> MRF: 3 ResBlock1 (k 3/7/11, dilations 1/3/5; leaky-ReLU
                 fused on the A operand, residual fused, the 1/3 average fused as
                 scale+accumulate)] x4 (rates 8,8,2,2) -> leaky-ReLU + conv_post k7
                 + tanh -> PCM16 written by the conv epilogue
Sample rate 22 050 Hz, hop 256.
"""
from __future__ import annotations

import math

import torch

from .. import ops
from .configs import VitsConfig

SYMBOLS = ("_;:,.!?¡¿—…\"«»“” " + "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz"
           + "ɑɐɒæɓʙβɔɕçɗɖðʤəɘɚɛɜɝɞɟʄɡɠɢʛɦɧħɥʜɨɪʝɭɬɫɮʟɱɯɰŋɳɲɴøɵɸθœɶʘ"
             + "ɹɺɾɻʀʁɽʂʃʈʧʉʊʋⱱʌɣɤʍχʎʏʑʐʒʔʡʕʢǀǁǂǃˈˌːˑʼʴʰʱʲʷˠˤ˞↓↑→↗↘'̩'ᵻ")


def text_to_ids(text: str, n_symbols: int, vocab: dict | None = None) -> list[int]:
    """Character-level symbol ids with VITS's blank interspersing (id 0).
    ``vocab`` (a checkpoint's vocab.json, character -> id): lower-cased text,
    characters outside it dropped, as the MMS-TTS character tokenizers do."""
    if vocab is not None:
        ids = [vocab[c] for c in text.lower() if c in vocab]
    else:
        table = {c: i for i, c in enumerate(SYMBOLS[:n_symbols])}
        ids = [table.get(c, table[" "]) for c in text]
    out = [0]
    for i in ids:
        out += [i, 0]
    return out


def _rnd(g, device, *shape, std=0.02):
    t = torch.empty(*shape, dtype=torch.float32, device=device)
    t.normal_(0.0, std, generator=g)
    return t.to(torch.bfloat16)


class VitsWeights:
    def __init__(self, cfg: VitsConfig, device, seed: int = 0):
        self.cfg = cfg
        dev = torch.device(device)
        g = torch.Generator(device=dev)
        g.manual_seed(seed * 7919 + 11)
        H, F, C = cfg.hidden, cfg.filter_channels, cfg.inter_channels
        zeros = lambda n: torch.zeros(n, dtype=torch.bfloat16, device=dev)  # noqa: E731
        ones = lambda n: torch.ones(n, dtype=torch.bfloat16, device=dev)   # noqa: E731
        # fan-in scaled random init keeps activations O(1) through the deep
        # stacks (a fixed small std would make the random-init waveform vanish)
        conv = lambda co, ci, k, std=None, gated=False: ops.ConvWeight(  # noqa: E731
            _rnd(g, dev, co, ci, k, std=(ci * k) ** -0.5 if std is None else std), zeros(co),
            gated=gated)
        self.emb = _rnd(g, dev, cfg.n_symbols, H, std=H ** -0.5)
        dh = H // cfg.n_heads
        self.enc = []
        for _ in range(cfg.enc_layers):
            self.enc.append({
                "qkv": conv(3 * H, H, 1), "o": conv(H, H, 1),
                "emb_k": _rnd(g, dev, 2 * cfg.window + 1, dh, std=dh ** -0.5),
                "emb_v": _rnd(g, dev, 2 * cfg.window + 1, dh, std=dh ** -0.5),
                "ln1_w": ones(H), "ln1_b": zeros(H),
                "ffn1": conv(F, H, cfg.kernel_size), "ffn2": conv(H, F, cfg.kernel_size),
                "ln2_w": ones(H), "ln2_b": zeros(H)})
        self.proj = conv(2 * C, H, 1)
        Fd = 256 if H >= 192 else H
        self.dp = {"c1": conv(Fd, H, 3), "ln1_w": ones(Fd), "ln1_b": zeros(Fd),
                   "c2": conv(Fd, Fd, 3), "ln2_w": ones(Fd), "ln2_b": zeros(Fd),
                   "proj": conv(1, Fd, 1)}
        half = C // 2
        self.flows = []
        for _ in range(cfg.flow_layers):
            wn = []
            for i in range(cfg.wn_layers):
                last = i == cfg.wn_layers - 1
                wn.append({"in": conv(2 * H, H, 5, gated=True),
                           "res": None if last else conv(H, H, 1),
                           "skip": conv(H, H, 1)})
            self.flows.append({"pre": conv(H, half, 1), "wn": wn,
                               "post": conv(half, H, 1, std=0.0)})   # VITS zero-inits post
        U = cfg.upsample_initial
        self.conv_pre = conv(U, C, 7)
        self.ups, self.res = [], []
        ch = U
        for i, r in enumerate(cfg.upsample_rates):
            k = 2 * r if r > 2 else 4
            co = ch // 2
            self.ups.append(ops.ConvTransposeWeight(_rnd(g, dev, ch, co, k, std=(ch * k / r) ** -0.5),
                                                    zeros(co),
                                                    r, (k - r) // 2))
            blocks = []
            for ks, dils in zip(cfg.resblock_kernels, cfg.resblock_dilations):
                blocks.append([(conv(co, co, ks), conv(co, co, ks), d) for d in dils])
            self.res.append(blocks)
            ch = co
        self.conv_post = ops.ConvWeight(_rnd(g, dev, 1, ch, 7, std=(ch * 7) ** -0.5), None)
        self.last_channels = ch
        self.sdp = None          # checkpoints: the stochastic duration predictor (loader)


class VitsModel:
    NOISE_SCALE = 0.667
    MAX_FRAMES_PER_SYMBOL = 12
    MAX_SDP_FRAMES = 100

    def __init__(self, w: VitsWeights):
        self.w = w
        self.cfg = w.cfg
        self._sdp = None
        if getattr(w, "sdp", None) is not None:
            from .vits_sdp import StochasticDurationPredictor
            self._sdp = StochasticDurationPredictor(w.sdp, kernel=w.cfg.sdp_kernel,
                                                    bins=w.cfg.sdp_bins, tail=w.cfg.sdp_tail)
        # random-init voice: the VITS default; checkpoints: their config's
        self.noise_scale = (w.cfg.noise_scale if getattr(w, "from_checkpoint", False)
                            else self.NOISE_SCALE)
        self.noise_scale_duration = w.cfg.noise_scale_duration
        self.spk = getattr(w, "spk", None)        # multi-speaker conditioning (loader)

    @property
    def n_speakers(self) -> int:
        return self.cfg.n_speakers if self.spk is not None else 1

    def speaker_vec(self, spk: torch.Tensor | None) -> torch.Tensor | None:
        """Speaker ids [B] (int64, device) -> embeddings g [B, gin] f32; None
        for single-speaker voices."""
        if self.spk is None:
            return None
        if spk is None:
            raise ValueError("a multi-speaker voice needs speaker ids")
        return self.spk["emb"][spk].float()

    def _proj(self, key, g: torch.Tensor, i: int | None = None) -> torch.Tensor:
        wgt, b = self.spk[key] if i is None else self.spk[key][i]
        return torch.nn.functional.linear(g, wgt, b)

    # ------------------------------------------------------------------ text
    def encode_text(self, ids: torch.Tensor, lens: torch.Tensor) -> torch.Tensor:
        """ids [B, T] int64 -> stats [B, T, 2C] (m_p | logs_p)."""
        cfg, w = self.cfg, self.w
        H = cfg.hidden
        dh = H // cfg.n_heads
        x = (w.emb[ids].float() * math.sqrt(H)).to(torch.bfloat16)
        T = ids.shape[1]
        mask = (torch.arange(T, device=ids.device)[None, :] < lens[:, None].long())[..., None]
        x = (x * mask).contiguous()
        for L in w.enc:
            qkv = ops.conv1d(x, L["qkv"], lens=lens)
            a = ops.relpos_attention(qkv, L["emb_k"], L["emb_v"], lens, cfg.n_heads, dh,
                                     cfg.window)
            y = ops.conv1d(a, L["o"], res=x, lens=lens)                       # x + attn
            x = ops.layernorm(y.view(-1, H), L["ln1_w"], L["ln1_b"], 1e-5).view_as(y)
            x = x * mask          # the FFN conv reads its neighbours: padded rows zero
            f = ops.conv1d(x, L["ffn1"], act="relu", lens=lens)
            y = ops.conv1d(f, L["ffn2"], res=x, lens=lens)
            x = ops.layernorm(y.view(-1, H), L["ln2_w"], L["ln2_b"], 1e-5).view_as(y)
            x = (x * mask).contiguous()
        return ops.conv1d(x, w.proj, lens=lens), x

    def durations(self, x: torch.Tensor, lens: torch.Tensor, length_scale: float = 1.0,
                  g: torch.Tensor | None = None) -> torch.Tensor:
        if self._sdp is not None:
            return self._sdp_durations(x, lens, length_scale, g)
        d = self.w.dp
        Fd = d["c1"].Cout
        T = x.shape[1]
        mask = (torch.arange(T, device=x.device)[None, :] < lens[:, None].long())[..., None]
        if g is not None:     # the speaker term on the predictor's input
            x = ((x.float() + self._proj("dp", g)[:, None, :]) * mask).to(torch.bfloat16)
        h = ops.conv1d(x, d["c1"], act="relu", lens=lens)
        h = ops.layernorm(h.view(-1, Fd), d["ln1_w"], d["ln1_b"], 1e-5).view_as(h) * mask
        h = ops.conv1d(h, d["c2"], act="relu", lens=lens)
        h = ops.layernorm(h.view(-1, Fd), d["ln2_w"], d["ln2_b"], 1e-5).view_as(h)
        logw = ops.conv1d(h, d["proj"], lens=lens)[..., 0].float()
        dur = torch.ceil(torch.exp(logw) * length_scale / self.cfg.speaking_rate)
        if not getattr(self.w, "from_checkpoint", False):
            dur = dur.clamp(1, self.MAX_FRAMES_PER_SYMBOL)
        T = x.shape[1]
        valid = torch.arange(T, device=x.device)[None, :] < lens[:, None].long()
        return (dur * valid).to(torch.int32)

    def _sdp_durations(self, x: torch.Tensor, lens: torch.Tensor, length_scale,
                       g: torch.Tensor | None = None) -> torch.Tensor:
        """Checkpoint voices: frames per symbol from the stochastic duration
        predictor, ceil(exp(log w) * length_scale), as the published models
        (no clamp; an all-zero phrase gets one frame)."""
        B, T, _ = x.shape
        mask = torch.arange(T, device=x.device)[None, :] < lens[:, None].long()
        noise = torch.randn(B, 2, T, device=x.device) * self.noise_scale_duration
        logw = self._sdp.log_durations(x, mask, noise,
                                       None if g is None else self._proj("dp", g))
        ls = length_scale / self.cfg.speaking_rate
        # guard only (a trained predictor stays far below it): one symbol may
        # not claim more than MAX_SDP_FRAMES frames (~1.6 s at 16 kHz / hop 256)
        dur = torch.ceil(torch.exp(logw) * ls).clamp(max=self.MAX_SDP_FRAMES) * mask
        first = (dur.sum(1, keepdim=True) == 0) & mask[:, :1]
        dur[:, :1] = torch.where(first, torch.ones_like(dur[:, :1]), dur[:, :1])
        return dur.to(torch.int32)

    # ------------------------------------------------------------------ flow
    def flow_reverse(self, z: torch.Tensor, flen: torch.Tensor,
                     g: torch.Tensor | None = None) -> torch.Tensor:
        cfg, w = self.cfg, self.w
        half, H = cfg.inter_channels // 2, cfg.hidden
        nf = len(w.flows)
        for k, fl in enumerate(reversed(w.flows)):
            z = z.flip(-1).contiguous()          # Flip (its own inverse)
            x0, x1 = z[..., :half], z[..., half:]
            h = ops.conv1d(x0, fl["pre"], lens=flen)
            skip = None
            gc = None if g is None else self._proj("flows", g, nf - 1 - k)   # [B, 2H * layers]
            for li, layer in enumerate(fl["wn"]):
                if gc is None:
                    acts = ops.conv1d(h, layer["in"], act="gated", lens=flen)
                else:
                    # multi-speaker: the speaker term enters between the conv
                    # and the gate, so the fused gate epilogue is not used
                    a = ops.conv1d(h, layer["in_plain"], lens=flen).float()
                    a = a + gc[:, None, 2 * H * li:2 * H * (li + 1)]
                    acts = (torch.tanh(a[..., :H]) * torch.sigmoid(a[..., H:])).to(torch.bfloat16)
                skip = ops.conv1d(acts, layer["skip"], acc=skip, lens=flen)   # skip += conv
                if layer["res"] is not None:
                    h = ops.conv1d(acts, layer["res"], res=h, lens=flen)      # h += conv
            # mean-only coupling, reverse: x1 <- x1 - post(skip), written in place
            ops.conv1d(skip, fl["post"], alpha=-1.0, acc=x1, out=x1, lens=flen)
        return z

    # --------------------------------------------------------------- decoder
    def decode(self, z: torch.Tensor, pcm_lens: torch.Tensor | None = None,
               g: torch.Tensor | None = None) -> torch.Tensor:
        """z [B, F, C] -> PCM16 [B, F * hop]."""
        w, cfg = self.w, self.cfg
        sl = cfg.leaky_slope
        x = ops.conv1d(z, w.conv_pre)
        if g is not None:
            x = (x.float() + self._proj("dec", g)[:, None, :]).to(torch.bfloat16)
        for i, ct in enumerate(w.ups):
            x = ops.conv_transpose1d(x, ct, pre_slope=sl)
            xs = None
            nb = len(w.res[i])
            for blocks in w.res[i]:
                xb = x
                for j, (c1, c2, d) in enumerate(blocks):
                    t = ops.conv1d(xb, c1, dil=d, pre_slope=sl)
                    if j < len(blocks) - 1:
                        xb = ops.conv1d(t, c2, pre_slope=sl, res=xb)
                    else:  # last pair of the block: xs += (conv + xb) / nb
                        xs = ops.conv1d(t, c2, pre_slope=sl, res=xb, alpha=1.0 / nb, acc=xs,
                                        out=xs)
            x = xs
        pcm = ops.conv1d(x, w.conv_post, pre_slope=0.01, act="tanh", pcm16=True, lens=pcm_lens)
        return pcm[..., 0]

    # ---------------------------------------------------------------- full
    def text_phase(self, ids: torch.Tensor, lens: torch.Tensor, length_scale,
                   spk: torch.Tensor | None = None
                   ) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        """Text encoder + durations -> (stats, cum, flen); ``length_scale`` a
        float or a device scalar (graph replay); ``spk`` speaker ids [B]
        (multi-speaker voices)."""
        stats, x = self.encode_text(ids, lens)
        dur = self.durations(x, lens, length_scale, self.speaker_vec(spk))
        cum = torch.cumsum(dur, dim=1, dtype=torch.int32).contiguous()
        return stats, cum, cum[:, -1].contiguous()

    def audio_phase(self, stats: torch.Tensor, cum: torch.Tensor, flen: torch.Tensor, F: int,
                    seed: int = 0, seed_dev: torch.Tensor | None = None,
                    spk: torch.Tensor | None = None) -> torch.Tensor:
        """Prior sample over F frames + reverse flow + vocoder -> PCM16 [B, F * hop]."""
        g = self.speaker_vec(spk)
        z = ops.expand_sample(stats, cum, flen, F, self.noise_scale, seed, seed_dev=seed_dev)
        z = self.flow_reverse(z, flen, g)
        return self.decode(z, (flen * self.hop).to(torch.int32), g)

    @property
    def hop(self) -> int:
        return int(math.prod(self.cfg.upsample_rates))

    def synthesize(self, ids: torch.Tensor, lens: torch.Tensor, *, seed: int = 0,
                   length_scale: float = 1.0, frame_step: int = 1,
                   speakers: torch.Tensor | None = None) -> tuple[torch.Tensor, torch.Tensor]:
        """ids [B, T] -> (PCM16 [B, S], samples per utterance [B]). The frame
        count is rounded up to ``frame_step`` (the graph runner's buckets).
        ``speakers``: speaker ids [B] of a multi-speaker voice."""
        stats, cum, flen = self.text_phase(ids, lens, length_scale, speakers)
        F = int(flen.max().item())
        F = -(-F // frame_step) * frame_step
        return self.audio_phase(stats, cum, flen, F, seed, spk=speakers), flen * self.hop


class VitsGraphRunner:
    """``VitsModel.synthesize`` as two HIP-graph replays per shape bucket.

    The frame count is data-dependent (predicted durations), so a synthesis is
    cut where the host must learn it: graph 1 (text encoder + durations) per
    (batch, symbols) bucket, one host read of the longest frame count, then
    graph 2 (prior sample + reverse flow + HiFi-GAN vocoder) per (batch,
    symbols, frames) bucket. ~190 eager launches become 2 replays, so a phrase
    batch holds the GIL for microseconds instead of milliseconds beside the
    decoder schedulers. Padding is inert: every stage masks by ``lens`` /
    ``flen``, rows are independent, and the prior noise of a frame does not
    depend on the padded frame count, so a bucketed replay gives the rows of
    the eager ``synthesize(..., frame_step=F_STEP)``. The seed and the length
    scale are device scalars written before each replay. Buckets are captured
    lazily into ONE memory pool; replays are serialised by the caller (the TTS
    engine's GPU lock), every call runs graph 1 then graph 2 of the same
    (batch, symbols) bucket, and graph 1's outputs stay alive, so no later
    capture can hand out their memory."""
    B_BUCKETS = (1, 2, 4, 8, 16, 32)
    T_STEP = 64
    F_STEP = 128
    MAX_AUDIO_GRAPHS = 48      # least recently used audio graphs beyond this are dropped

    def __init__(self, model: VitsModel, device, *, max_symbols: int = 512, max_frames: int = 4096):
        import collections
        self.model = model
        self.device = torch.device(device)
        self.max_symbols = max_symbols
        self.max_frames = max_frames
        self.pool = torch.cuda.graph_pool_handle()
        self._text: dict = {}
        # LRU: each audio graph keeps its PCM output (up to tens of MB) alive
        self._audio: collections.OrderedDict = collections.OrderedDict()
        self.stats = {"replays": 0, "captures": 0, "eager": 0, "evicted": 0}

    def _bucket_b(self, B: int) -> int | None:
        for b in self.B_BUCKETS:
            if B <= b:
                return b
        return None

    def _capture(self, fn):
        st = torch.cuda.current_stream(self.device)
        fn()                       # warm-up outside the graph (kernels, allocator)
        st.synchronize()
        g = torch.cuda.CUDAGraph()
        # the placed TTS stream (never a new pool stream: utils/streams.py);
        # thread-local capture: the decoder threads keep launching meanwhile
        with torch.cuda.graph(g, pool=self.pool, stream=st, capture_error_mode="thread_local"):
            out = fn()
        self.stats["captures"] += 1
        return g, out

    def _text_graph(self, Bb: int, Tb: int):
        ent = self._text.get((Bb, Tb))
        if ent is None:
            ids = torch.zeros(Bb, Tb, dtype=torch.int64, device=self.device)
            lens = torch.ones(Bb, dtype=torch.int32, device=self.device)
            ls = torch.ones(1, dtype=torch.float32, device=self.device)
            spk = (torch.zeros(Bb, dtype=torch.int64, device=self.device)
                   if self.model.n_speakers > 1 else None)
            g, out = self._capture(lambda: self.model.text_phase(ids, lens, ls, spk))
            ent = self._text[(Bb, Tb)] = (g, ids, lens, ls, out, spk)
        return ent

    def _audio_graph(self, Bb: int, Tb: int, Fb: int, text_out, spk):
        key = (Bb, Tb, Fb)
        ent = self._audio.get(key)
        if ent is None:
            while len(self._audio) >= self.MAX_AUDIO_GRAPHS:
                # the graph and its tensors go back to the shared pool; its text
                # graph (whose outputs it reads) stays, text graphs are few
                self._audio.popitem(last=False)
                self.stats["evicted"] += 1
            seed = torch.zeros(1, dtype=torch.int32, device=self.device)
            stats, cum, flen = text_out
            g, pcm = self._capture(lambda: self.model.audio_phase(stats, cum, flen, Fb,
                                                                  seed_dev=seed, spk=spk))
            ent = self._audio[key] = (g, seed, pcm)
        else:
            self._audio.move_to_end(key)
        return ent

    def synthesize(self, ids: torch.Tensor, lens: torch.Tensor, *, seed: int = 0,
                   length_scale: float = 1.0, speakers: torch.Tensor | None = None
                   ) -> tuple[torch.Tensor, torch.Tensor]:
        """As ``VitsModel.synthesize``; shapes outside the buckets run eagerly.
        ``speakers``: device speaker ids [B] (multi-speaker voices; written
        into the bucket's id buffer before the replays)."""
        B, T = ids.shape
        Bb = self._bucket_b(B)
        Tb = -(-T // self.T_STEP) * self.T_STEP
        if Bb is None or Tb > self.max_symbols:
            self.stats["eager"] += 1
            return self.model.synthesize(ids, lens, seed=seed, length_scale=length_scale,
                                         frame_step=self.F_STEP, speakers=speakers)
        g1, s_ids, s_lens, s_ls, text_out, s_spk = self._text_graph(Bb, Tb)
        s_ids.zero_()
        s_ids[:B, :T].copy_(ids)
        s_lens.fill_(1)
        s_lens[:B].copy_(lens)
        s_ls.fill_(float(length_scale))
        if s_spk is not None:
            s_spk.zero_()
            if speakers is not None:
                s_spk[:B].copy_(speakers)
        g1.replay()
        stats, cum, flen = text_out
        F = int(flen[:B].max().item())
        Fb = -(-F // self.F_STEP) * self.F_STEP
        if Fb > self.max_frames:
            self.stats["eager"] += 1
            pcm = self.model.audio_phase(stats[:B], cum[:B], flen[:B].contiguous(), Fb, seed,
                                         spk=None if s_spk is None else s_spk[:B])
            return pcm, flen[:B] * self.model.hop
        g2, s_seed, pcm = self._audio_graph(Bb, Tb, Fb, text_out, s_spk)
        s_seed.fill_(seed & 0x7FFFFFFF)
        g2.replay()
        self.stats["replays"] += 1
        return pcm[:B], flen[:B] * self.model.hop
