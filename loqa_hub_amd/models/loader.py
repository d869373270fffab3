"""Checkpoint I/O (SURVEY §5.4 "New"): safetensors mmap -> pinned host ->
device, in the Hugging Face tensor naming of the public Whisper and Llama
checkpoints, plus the data-parallel weight broadcast.

The reference has no model weights at all (inference lives in external
services); BASELINE runs use seeded random init, which every rank reproduces
locally without communication. Real checkpoints go through here:

* ``load_llama`` / ``load_whisper``: read a safetensors file (or a directory
  of shards) with ``safe_open`` (memory-mapped: nothing is unpickled, nothing
  executes), stage each tensor through pinned memory and copy it to the device
  with a non-blocking H2D copy, then assemble the framework's fused layouts
  (q|k|v and gate|up row blocks, the Whisper conv as [Cout, Cin*3]).
* ``save_llama`` / ``save_whisper``: the inverse mapping (round-trip tests,
  exporting fine-tuned weights).
* ``broadcast_state``: rank 0 holds the tensors; every other rank receives
  them in ~256 MB flat buckets over ``torch.distributed`` (RCCL over xGMI on
  the GPUs: a few large collectives instead of one per tensor).
"""
from __future__ import annotations

import glob
import os

import torch

from .configs import LlamaConfig, WhisperConfig
from .llama import LlamaWeights, TPGroup
from .whisper import WhisperWeights, sinusoids

BUCKET_BYTES = 256 << 20


# ------------------------------------------------------------------- file I/O
def _files(path: str) -> list[str]:
    if os.path.isdir(path):
        fs = sorted(glob.glob(os.path.join(path, "*.safetensors")))
        if not fs:
            raise FileNotFoundError(f"no *.safetensors under {path}")
        return fs
    return [path]


def read_safetensors(path: str, device, dtype=torch.bfloat16) -> dict[str, torch.Tensor]:
    """All tensors of a checkpoint on ``device`` (floating tensors cast to
    ``dtype``); host staging is pinned so the H2D copies are asynchronous."""
    from safetensors import safe_open
    dev = torch.device(device)
    out: dict[str, torch.Tensor] = {}
    for f in _files(path):
        with safe_open(f, framework="pt", device="cpu") as st:
            for name in st.keys():
                t = st.get_tensor(name)
                if t.is_floating_point():
                    t = t.to(dtype)
                if dev.type == "cuda":
                    t = t.pin_memory().to(dev, non_blocking=True)
                out[name] = t.contiguous()
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    return out


def write_safetensors(state: dict[str, torch.Tensor], path: str) -> None:
    from safetensors.torch import save_file
    save_file({k: v.detach().contiguous().cpu() for k, v in state.items()}, path)


# ---------------------------------------------------------------------- Llama
def llama_state_dict(w: LlamaWeights) -> dict[str, torch.Tensor]:
    """Hugging Face ``LlamaForCausalLM`` names of an unsharded model."""
    cfg = w.cfg
    H, Hkv, D, F = cfg.n_heads, cfg.n_kv_heads, cfg.head_dim, cfg.ffn_dim
    sd = {"model.embed_tokens.weight": w.embed, "model.norm.weight": w.final_norm}
    if not cfg.tie_embeddings:
        sd["lm_head.weight"] = w.lm_head
    for i, L in enumerate(w.layers):
        p = f"model.layers.{i}."
        q, k, v = L["wqkv"].split([H * D, Hkv * D, Hkv * D])
        g, u = L["w_gate_up"].split([F, F])
        sd.update({p + "input_layernorm.weight": L["attn_norm"],
                   p + "self_attn.q_proj.weight": q, p + "self_attn.k_proj.weight": k,
                   p + "self_attn.v_proj.weight": v, p + "self_attn.o_proj.weight": L["wo"],
                   p + "post_attention_layernorm.weight": L["mlp_norm"],
                   p + "mlp.gate_proj.weight": g, p + "mlp.up_proj.weight": u,
                   p + "mlp.down_proj.weight": L["w_down"]})
    return sd


def llama_from_state_dict(cfg: LlamaConfig, sd: dict[str, torch.Tensor], device,
                          tp: TPGroup | None = None) -> LlamaWeights:
    layers = []
    for i in range(cfg.n_layers):
        p = f"model.layers.{i}."
        layers.append({
            "attn_norm": sd[p + "input_layernorm.weight"],
            "wqkv": torch.cat([sd[p + "self_attn.q_proj.weight"], sd[p + "self_attn.k_proj.weight"],
                               sd[p + "self_attn.v_proj.weight"]]).contiguous(),
            "wo": sd[p + "self_attn.o_proj.weight"],
            "mlp_norm": sd[p + "post_attention_layernorm.weight"],
            "w_gate_up": torch.cat([sd[p + "mlp.gate_proj.weight"],
                                    sd[p + "mlp.up_proj.weight"]]).contiguous(),
            "w_down": sd[p + "mlp.down_proj.weight"]})
    return LlamaWeights.from_tensors(cfg, device, embed=sd["model.embed_tokens.weight"],
                                     layers=layers, final_norm=sd["model.norm.weight"],
                                     lm_head=sd.get("lm_head.weight"), tp=tp)


def save_llama(w: LlamaWeights, path: str) -> None:
    write_safetensors(llama_state_dict(w), path)


def load_llama(cfg: LlamaConfig, path: str, device, tp: TPGroup | None = None) -> LlamaWeights:
    return llama_from_state_dict(cfg, read_safetensors(path, device), device, tp)


# -------------------------------------------------------------------- Whisper
def _split_qkv(L: dict, d: int, pre: str, sd: dict, cross: bool) -> None:
    if cross:
        sd[pre + "q_proj.weight"], sd[pre + "q_proj.bias"] = L["xq"], L["xq_b"]
        k, v = L["xkv"].split([d, d])
        kb, vb = L["xkv_b"].split([d, d])
        sd[pre + "k_proj.weight"], sd[pre + "v_proj.weight"], sd[pre + "v_proj.bias"] = k, v, vb
        sd[pre + "out_proj.weight"], sd[pre + "out_proj.bias"] = L["xo"], L["xo_b"]
        return
    q, k, v = L["wqkv"].split([d, d, d])
    qb, _, vb = L["bqkv"].split([d, d, d])
    sd.update({pre + "q_proj.weight": q, pre + "q_proj.bias": qb, pre + "k_proj.weight": k,
               pre + "v_proj.weight": v, pre + "v_proj.bias": vb,
               pre + "out_proj.weight": L["wo"], pre + "out_proj.bias": L["bo"]})


def whisper_state_dict(w: WhisperWeights) -> dict[str, torch.Tensor]:
    """Hugging Face ``WhisperForConditionalGeneration`` names."""
    cfg, d = w.cfg, w.cfg.d_model
    M = cfg.n_mels
    sd = {"model.encoder.conv1.weight": w.conv1_w.view(d, M, 3),
          "model.encoder.conv1.bias": w.conv1_b,
          "model.encoder.conv2.weight": w.conv2_w.view(d, d, 3),
          "model.encoder.conv2.bias": w.conv2_b,
          "model.encoder.embed_positions.weight": w.pos_enc,
          "model.encoder.layer_norm.weight": w.enc_ln_w,
          "model.encoder.layer_norm.bias": w.enc_ln_b,
          "model.decoder.embed_tokens.weight": w.tok_embed,
          "model.decoder.embed_positions.weight": w.dec_pos,
          "model.decoder.layer_norm.weight": w.dec_ln_w,
          "model.decoder.layer_norm.bias": w.dec_ln_b}
    for side, blocks in (("encoder", w.enc), ("decoder", w.dec)):
        for i, L in enumerate(blocks):
            p = f"model.{side}.layers.{i}."
            _split_qkv(L, d, p + "self_attn.", sd, cross=False)
            sd.update({p + "self_attn_layer_norm.weight": L["ln1_w"],
                       p + "self_attn_layer_norm.bias": L["ln1_b"],
                       p + "fc1.weight": L["fc1"], p + "fc1.bias": L["fc1_b"],
                       p + "fc2.weight": L["fc2"], p + "fc2.bias": L["fc2_b"],
                       p + "final_layer_norm.weight": L["ln2_w"],
                       p + "final_layer_norm.bias": L["ln2_b"]})
            if side == "decoder":
                _split_qkv(L, d, p + "encoder_attn.", sd, cross=True)
                sd[p + "encoder_attn_layer_norm.weight"] = L["lnx_w"]
                sd[p + "encoder_attn_layer_norm.bias"] = L["lnx_b"]
    return sd


def whisper_from_state_dict(cfg: WhisperConfig, sd: dict[str, torch.Tensor],
                            device) -> WhisperWeights:
    d = cfg.d_model
    dev = torch.device(device)
    some = sd["model.decoder.embed_tokens.weight"]

    def zeros(n):
        return torch.zeros(n, dtype=some.dtype, device=some.device)

    def block(p: str, cross: bool) -> dict:
        a = p + "self_attn."
        b = {"ln1_w": sd[p + "self_attn_layer_norm.weight"],
             "ln1_b": sd[p + "self_attn_layer_norm.bias"],
             "wqkv": torch.cat([sd[a + "q_proj.weight"], sd[a + "k_proj.weight"],
                                sd[a + "v_proj.weight"]]).contiguous(),
             "bqkv": torch.cat([sd[a + "q_proj.bias"], sd.get(a + "k_proj.bias", zeros(d)),
                                sd[a + "v_proj.bias"]]).contiguous(),
             "wo": sd[a + "out_proj.weight"], "bo": sd[a + "out_proj.bias"],
             "ln2_w": sd[p + "final_layer_norm.weight"], "ln2_b": sd[p + "final_layer_norm.bias"],
             "fc1": sd[p + "fc1.weight"], "fc1_b": sd[p + "fc1.bias"],
             "fc2": sd[p + "fc2.weight"], "fc2_b": sd[p + "fc2.bias"]}
        if cross:
            x = p + "encoder_attn."
            b.update({"lnx_w": sd[p + "encoder_attn_layer_norm.weight"],
                      "lnx_b": sd[p + "encoder_attn_layer_norm.bias"],
                      "xq": sd[x + "q_proj.weight"], "xq_b": sd[x + "q_proj.bias"],
                      "xkv": torch.cat([sd[x + "k_proj.weight"],
                                        sd[x + "v_proj.weight"]]).contiguous(),
                      "xkv_b": torch.cat([sd.get(x + "k_proj.bias", zeros(d)),
                                          sd[x + "v_proj.bias"]]).contiguous(),
                      "xo": sd[x + "out_proj.weight"], "xo_b": sd[x + "out_proj.bias"]})
        return b

    pos = sd.get("model.encoder.embed_positions.weight")
    if pos is None:
        pos = sinusoids(cfg.n_audio_ctx, d).to(device=dev, dtype=some.dtype)
    return WhisperWeights.from_tensors(
        cfg,
        conv1_w=sd["model.encoder.conv1.weight"].reshape(d, -1).contiguous(),
        conv1_b=sd["model.encoder.conv1.bias"],
        conv2_w=sd["model.encoder.conv2.weight"].reshape(d, -1).contiguous(),
        conv2_b=sd["model.encoder.conv2.bias"], pos_enc=pos,
        enc=[block(f"model.encoder.layers.{i}.", False) for i in range(cfg.enc_layers)],
        enc_ln_w=sd["model.encoder.layer_norm.weight"], enc_ln_b=sd["model.encoder.layer_norm.bias"],
        tok_embed=sd["model.decoder.embed_tokens.weight"],
        dec_pos=sd["model.decoder.embed_positions.weight"],
        dec=[block(f"model.decoder.layers.{i}.", True) for i in range(cfg.dec_layers)],
        dec_ln_w=sd["model.decoder.layer_norm.weight"], dec_ln_b=sd["model.decoder.layer_norm.bias"])


def save_whisper(w: WhisperWeights, path: str) -> None:
    write_safetensors(whisper_state_dict(w), path)


def load_whisper(cfg: WhisperConfig, path: str, device) -> WhisperWeights:
    return whisper_from_state_dict(cfg, read_safetensors(path, device), device)


# ------------------------------------------------------------ D2: broadcast
def broadcast_state(state: dict[str, torch.Tensor] | None, src: int = 0, group=None,
                    device=None, bucket_bytes: int = BUCKET_BYTES) -> dict[str, torch.Tensor]:
    """Replicate ``state`` (present on rank ``src`` only) to every rank of
    ``group``: metadata as one object broadcast, the tensors packed into flat
    buckets of ``bucket_bytes`` per dtype, one ``broadcast`` per bucket."""
    import torch.distributed as dist
    rank = dist.get_rank(group)
    meta = [None]
    if rank == src:
        meta = [[(k, tuple(v.shape), str(v.dtype).replace("torch.", "")) for k, v in state.items()]]
    dist.broadcast_object_list(meta, src=src, group=group)
    items = meta[0]
    if device is None:
        device = next(iter(state.values())).device if rank == src else torch.device("cpu")
    out: dict[str, torch.Tensor] = {}
    by_dtype: dict[str, list] = {}
    for k, shape, dt in items:
        by_dtype.setdefault(dt, []).append((k, shape))
    for dt, entries in by_dtype.items():
        dtype = getattr(torch, dt)
        esz = torch.empty((), dtype=dtype).element_size()
        i = 0
        while i < len(entries):
            chunk, n = [], 0
            while i < len(entries):
                numel = 1
                for s in entries[i][1]:
                    numel *= s
                if chunk and (n + numel) * esz > bucket_bytes:
                    break
                chunk.append((entries[i][0], entries[i][1], numel))
                n += numel
                i += 1
            if rank == src:
                flat = torch.cat([state[k].reshape(-1).to(device) for k, _, _ in chunk])
            else:
                flat = torch.empty(n, dtype=dtype, device=device)
            dist.broadcast(flat, src=src, group=group)
            off = 0
            for k, shape, numel in chunk:
                out[k] = flat[off:off + numel].view(shape) if rank != src else state[k]
                off += numel
    return out


# ----------------------------------------------------------------------- VITS
def _wn(sd: dict, pre: str) -> torch.Tensor:
    """A conv weight, folding a weight-norm pair (``parametrizations.weight.
    original0/1`` or ``weight_g / weight_v``) into the plain weight:
    w = g * v / ||v|| with the norm over every dim but the first."""
    if pre + ".weight" in sd:
        return sd[pre + ".weight"].float()
    for g_key, v_key in ((".parametrizations.weight.original0", ".parametrizations.weight.original1"),
                         (".weight_g", ".weight_v")):
        if pre + g_key in sd:
            g, v = sd[pre + g_key].float(), sd[pre + v_key].float()
            n = v.flatten(1).norm(dim=1).view(-1, *([1] * (v.dim() - 1)))
            return g * v / n
    raise KeyError(pre + ".weight")


def _dds(sd: dict, pre: str) -> dict:
    layers = []
    i = 0
    while f"{pre}.convs_dilated.{i}.weight" in sd:
        layers.append({"dw_w": sd[f"{pre}.convs_dilated.{i}.weight"].float(),
                       "dw_b": sd[f"{pre}.convs_dilated.{i}.bias"].float(),
                       "pw_w": sd[f"{pre}.convs_pointwise.{i}.weight"].float(),
                       "pw_b": sd[f"{pre}.convs_pointwise.{i}.bias"].float(),
                       "n1_w": sd[f"{pre}.norms_1.{i}.weight"].float(),
                       "n1_b": sd[f"{pre}.norms_1.{i}.bias"].float(),
                       "n2_w": sd[f"{pre}.norms_2.{i}.weight"].float(),
                       "n2_b": sd[f"{pre}.norms_2.{i}.bias"].float()})
        i += 1
    return {"layers": layers}


def vits_from_state_dict(cfg, sd: dict[str, torch.Tensor], device):
    """``VitsWeights`` from a Hugging Face VITS / MMS-TTS state dict
    (``VitsModel`` naming; single or multi speaker). The training-only
    posterior encoder and the duration predictor's posterior flows are not
    read."""
    from . import vits as V
    from .. import ops
    if cfg.upsample_kernels and any(k % r for k, r in zip(cfg.upsample_kernels, cfg.upsample_rates)):
        raise ValueError("upsample kernel sizes must be multiples of their rates (polyphase form)")
    dev = torch.device(device)
    w = V.VitsWeights.__new__(V.VitsWeights)
    w.cfg = cfg
    f = lambda k: sd[k].float()                                   # noqa: E731
    bf = lambda t: t.to(torch.bfloat16) if t is not None else None  # noqa: E731
    conv = lambda wt, b=None, gated=False: ops.ConvWeight(bf(wt), bf(b), gated=gated)  # noqa: E731
    H = cfg.hidden
    w.emb = bf(f("text_encoder.embed_tokens.weight"))
    w.enc = []
    for i in range(cfg.enc_layers):
        p = f"text_encoder.encoder.layers.{i}."
        qkv_w = torch.cat([f(p + f"attention.{n}_proj.weight") for n in "qkv"])[:, :, None]
        qkv_b = torch.cat([f(p + f"attention.{n}_proj.bias") for n in "qkv"])
        w.enc.append({
            "qkv": conv(qkv_w, qkv_b),
            "o": conv(f(p + "attention.out_proj.weight")[:, :, None], f(p + "attention.out_proj.bias")),
            "emb_k": bf(f(p + "attention.emb_rel_k")[0]), "emb_v": bf(f(p + "attention.emb_rel_v")[0]),
            "ln1_w": bf(f(p + "layer_norm.weight")), "ln1_b": bf(f(p + "layer_norm.bias")),
            "ffn1": conv(f(p + "feed_forward.conv_1.weight"), f(p + "feed_forward.conv_1.bias")),
            "ffn2": conv(f(p + "feed_forward.conv_2.weight"), f(p + "feed_forward.conv_2.bias")),
            "ln2_w": bf(f(p + "final_layer_norm.weight")), "ln2_b": bf(f(p + "final_layer_norm.bias"))})
    w.proj = conv(f("text_encoder.project.weight"), f("text_encoder.project.bias"))
    dp = "duration_predictor."
    w.from_checkpoint = True          # durations unclamped, as the published models
    if cfg.sdp:
        # stochastic duration predictor (fp32: it runs at the symbol count)
        flows = [{"kind": "affine", "translate": f(dp + "flows.0.translate"),
                  "log_scale": f(dp + "flows.0.log_scale")}]
        for j in range(1, cfg.sdp_flows + 1):
            q = f"{dp}flows.{j}."
            flows.append({"kind": "conv", "pre_w": f(q + "conv_pre.weight"),
                          "pre_b": f(q + "conv_pre.bias"), "dds": _dds(sd, q + "conv_dds"),
                          "proj_w": f(q + "conv_proj.weight"), "proj_b": f(q + "conv_proj.bias")})
        w.sdp = {"pre_w": f(dp + "conv_pre.weight"), "pre_b": f(dp + "conv_pre.bias"),
                 "dds": _dds(sd, dp + "conv_dds"),
                 "proj_w": f(dp + "conv_proj.weight"), "proj_b": f(dp + "conv_proj.bias"),
                 "flows": flows}
        w.dp = None
    else:
        # deterministic predictor: (k conv + ReLU + LayerNorm) x2 -> 1x1, the
        # random-init voice's own structure
        w.sdp = None
        w.dp = {"c1": conv(f(dp + "conv_1.weight"), f(dp + "conv_1.bias")),
                "ln1_w": bf(f(dp + "norm_1.weight")), "ln1_b": bf(f(dp + "norm_1.bias")),
                "c2": conv(f(dp + "conv_2.weight"), f(dp + "conv_2.bias")),
                "ln2_w": bf(f(dp + "norm_2.weight")), "ln2_b": bf(f(dp + "norm_2.bias")),
                "proj": conv(f(dp + "proj.weight"), f(dp + "proj.bias"))}
    # prior flow: mean-only coupling layers over WaveNets
    w.flows = []
    for i in range(cfg.flow_layers):
        p = f"flow.flows.{i}."
        wn = []
        for j in range(cfg.wn_layers):
            last = j == cfg.wn_layers - 1
            rs_w, rs_b = _wn(sd, p + f"wavenet.res_skip_layers.{j}"), f(p + f"wavenet.res_skip_layers.{j}.bias")
            wn.append({"in": conv(_wn(sd, p + f"wavenet.in_layers.{j}"), f(p + f"wavenet.in_layers.{j}.bias"),
                                  gated=True),
                       "res": None if last else conv(rs_w[:H], rs_b[:H]),
                       "skip": conv(rs_w if last else rs_w[H:], rs_b if last else rs_b[H:])})
        w.flows.append({"pre": conv(f(p + "conv_pre.weight"), f(p + "conv_pre.bias")), "wn": wn,
                        "post": conv(f(p + "conv_post.weight"), f(p + "conv_post.bias"))})
    # speaker conditioning (multi-speaker checkpoints): the embedding table and
    # the 1x1 projections of a speaker vector g, applied per row (fp32, tiny)
    w.spk = None
    if cfg.n_speakers > 1:
        lin = lambda pre: (_wn(sd, pre)[:, :, 0].contiguous(), f(pre + ".bias"))  # noqa: E731
        w.spk = {"emb": f("embed_speaker.weight"), "dp": lin(dp + "cond"),
                 "flows": [lin(f"flow.flows.{i}.wavenet.cond_layer") for i in range(cfg.flow_layers)],
                 "dec": lin("decoder.cond")}
        # the WaveNet input convs without the fused gate: the speaker term is
        # added between the conv and tanh / sigmoid
        for i, fl in enumerate(w.flows):
            p = f"flow.flows.{i}."
            for j, layer in enumerate(fl["wn"]):
                layer["in_plain"] = conv(_wn(sd, p + f"wavenet.in_layers.{j}"),
                                         f(p + f"wavenet.in_layers.{j}.bias"))
    # HiFi-GAN generator
    w.conv_pre = conv(_wn(sd, "decoder.conv_pre"), f("decoder.conv_pre.bias"))
    w.ups, w.res = [], []
    nk = len(cfg.resblock_kernels)
    for i, r in enumerate(cfg.upsample_rates):
        ut = _wn(sd, f"decoder.upsampler.{i}")
        k = ut.shape[2]
        w.ups.append(ops.ConvTransposeWeight(bf(ut), bf(f(f"decoder.upsampler.{i}.bias")), r, (k - r) // 2))
        blocks = []
        for j, dils in enumerate(cfg.resblock_dilations):
            rb = f"decoder.resblocks.{i * nk + j}."
            blocks.append([(conv(_wn(sd, rb + f"convs1.{m}"), f(rb + f"convs1.{m}.bias")),
                            conv(_wn(sd, rb + f"convs2.{m}"), f(rb + f"convs2.{m}.bias")), d)
                           for m, d in enumerate(dils)])
        w.res.append(blocks)
    w.conv_post = conv(_wn(sd, "decoder.conv_post"))
    w.last_channels = w.conv_post.Cin
    if dev.type != "cpu":
        torch.cuda.synchronize(dev)
    return w


def load_vits(path: str, device, cfg=None):
    """(VitsConfig, VitsWeights, vocab or None) of a Hugging Face VITS /
    MMS-TTS checkpoint directory (config.json + *.safetensors [+ vocab.json])."""
    import json
    from .configs import checkpoint_config, vits_config_from_hf
    if cfg is None:
        d = checkpoint_config(path)
        if d is None:
            raise FileNotFoundError(f"no config.json for the VITS checkpoint {path}")
        if d.get("wavenet_dilation_rate", 1) != 1:
            raise ValueError("only VITS with WaveNet dilation rate 1 is supported")
        cfg = vits_config_from_hf(d, os.path.basename(os.path.normpath(path)))
    sd = read_safetensors(path, device, dtype=torch.float32)
    vocab = None
    vf = os.path.join(path if os.path.isdir(path) else os.path.dirname(path), "vocab.json")
    if os.path.exists(vf):
        with open(vf, encoding="utf-8") as fh:
            vocab = json.load(fh)
    return cfg, vits_from_state_dict(cfg, sd, device), vocab
