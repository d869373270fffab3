"""Checkpoint I/O: safetensors round trips in the Hugging Face
naming for Llama and Whisper (same tensors, same model outputs), and the
data-parallel weight broadcast (D2) over gloo with 2 ranks."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from loqa_hub_amd.models import loader
from loqa_hub_amd.models.configs import llama_config, whisper_config


def test_llama_safetensors_roundtrip(tmp_path):
    from loqa_hub_amd.models.llama import LlamaWeights
    cfg = llama_config("test-tiny")
    w = LlamaWeights(cfg, "cpu", seed=5)
    path = str(tmp_path / "llama.safetensors")
    loader.save_llama(w, path)
    w2 = loader.load_llama(cfg, path, "cpu")
    assert torch.equal(w.embed, w2.embed) and torch.equal(w.final_norm, w2.final_norm)
    for a, b in zip(w.layers, w2.layers):
        for k in a:
            assert torch.equal(a[k], b[k]), k
    for a, b in zip(w.decode_layers, w2.decode_layers):
        assert torch.equal(a["wqkv_f"], b["wqkv_f"]) and torch.equal(a["w_down"], b["w_down"])
    sd = loader.llama_state_dict(w2)
    assert "model.layers.0.self_attn.k_proj.weight" in sd
    assert sd["model.layers.0.mlp.gate_proj.weight"].shape == (cfg.ffn_dim, cfg.d_model)


def test_whisper_safetensors_roundtrip(tmp_path):
    from loqa_hub_amd.models.whisper import WhisperModel, WhisperWeights
    cfg = whisper_config("test-whisper")
    w = WhisperWeights(cfg, "cpu", seed=2)
    path = str(tmp_path / "whisper.safetensors")
    loader.save_whisper(w, path)
    w2 = loader.load_whisper(cfg, path, "cpu")
    for a, b in zip(w.dec + w.enc, w2.dec + w2.enc):
        for k in a:
            assert torch.equal(a[k], b[k]), k
    audio = torch.randn(1, 480000) * 0.1
    e1, e2 = WhisperModel(w).encode(audio), WhisperModel(w2).encode(audio)
    assert torch.equal(e1, e2)


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _bcast_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        state = None
        if rank == 0:
            g = torch.Generator().manual_seed(0)
            state = {f"t{i}": torch.randn(97 * (i + 1), 3, generator=g).to(
                torch.bfloat16 if i % 2 else torch.float32) for i in range(7)}
            state["ids"] = torch.arange(11)
        got = loader.broadcast_state(state, bucket_bytes=4096)
        torch.save({k: v.clone() for k, v in got.items()}, os.path.join(out_dir, f"r{rank}.pt"))
    finally:
        dist.destroy_process_group()


def test_broadcast_state_gloo(tmp_path):
    mp.start_processes(_bcast_worker, args=(2, _port(), str(tmp_path)), nprocs=2, join=True,
                       start_method="spawn")
    a = torch.load(tmp_path / "r0.pt", weights_only=True)
    b = torch.load(tmp_path / "r1.pt", weights_only=True)
    assert a.keys() == b.keys() and len(a) == 8
    for k in a:
        assert a[k].dtype == b[k].dtype and torch.equal(a[k], b[k]), k


def test_checkpoint_config_json_cpu(tmp_path):
    """A checkpoint's config.json (Hugging Face keys) sets the model shape:
    Llama-3.2-style with llama3 RoPE scaling, and Whisper; GPUConfig prefers it
    over the named model."""
    import json as _json

    import pytest
    import math

    from loqa_hub_amd.config import GPUConfig
    from loqa_hub_amd.models.configs import (checkpoint_config, llama_config,
                                             llama_config_from_hf, whisper_config,
                                             whisper_config_from_hf)
    from loqa_hub_amd.ops.reference import rope_cos_sin
    d = {"hidden_size": 2048, "num_hidden_layers": 16, "num_attention_heads": 32,
         "num_key_value_heads": 8, "intermediate_size": 8192, "vocab_size": 128256,
         "rope_theta": 500000.0, "rms_norm_eps": 1e-5, "tie_word_embeddings": True,
         "max_position_embeddings": 131072,
         "rope_scaling": {"rope_type": "llama3", "factor": 32.0, "low_freq_factor": 1.0,
                          "high_freq_factor": 4.0, "original_max_position_embeddings": 8192}}
    c = llama_config_from_hf(d, "x")
    ref = llama_config("llama3.2-1b")
    for k in ("d_model", "n_layers", "n_heads", "n_kv_heads", "head_dim", "ffn_dim", "vocab_size",
              "rope_theta", "tie_embeddings", "rope_scaling"):
        assert getattr(c, k) == getattr(ref, k), k
    # scaled table: short wavelengths untouched, long ones slowed 32x
    plain = rope_cos_sin(64, 16, 500000.0)
    sc = rope_cos_sin(64, 16, 500000.0, scaling=c.rope_scaling)
    assert torch.equal(sc[:, 0], plain[:, 0])
    ang_p, ang_s = math.atan2(plain[1, -1, 1], plain[1, -1, 0]), math.atan2(sc[1, -1, 1], sc[1, -1, 0])
    assert abs(ang_s * 32 - ang_p) < 1e-6
    with pytest.raises(ValueError):
        llama_config_from_hf(dict(d, rope_scaling={"type": "yarn", "factor": 4.0}))
    w = {"num_mel_bins": 128, "d_model": 1280, "encoder_layers": 32, "decoder_layers": 32,
         "encoder_attention_heads": 20, "vocab_size": 51866, "encoder_ffn_dim": 5120,
         "max_source_positions": 1500, "max_target_positions": 448}
    assert whisper_config_from_hf(w, "whisper-large-v3") == whisper_config("whisper-large-v3")
    os.makedirs(tmp_path / "ck")
    with open(tmp_path / "ck" / "config.json", "w") as fh:
        _json.dump(d, fh)
    assert checkpoint_config(str(tmp_path / "ck")) == d
    assert checkpoint_config(str(tmp_path / "ck" / "model.safetensors")) == d
    assert checkpoint_config(str(tmp_path)) is None
    g = GPUConfig(llm_model="tinyllama", llm_checkpoint=str(tmp_path / "ck"))
    assert g.llm_config().d_model == 2048 and g.llm_config().rope_scaling == (32.0, 1.0, 4.0, 8192)
    assert GPUConfig(llm_model="tinyllama").llm_config() == llama_config("tinyllama")
    assert GPUConfig(stt_model="whisper-base").stt_config() == whisper_config("whisper-base")
