"""A checkpoint's own ``tokenizer.json`` behind the engines (``engine/tokenizer.py``
``HFTokenizer``): byte-level BPE (the Llama-3 / Whisper kind) and SentencePiece-
style Metaspace BPE (the TinyLlama / Llama-2 kind), both trained here from a
small corpus with the ``tokenizers`` library (no network, no downloaded
vocabulary). Parity of a real checkpoint's token ids is unpinned: none of the
reference's files hold a tokenizer."""
import json
import os

import pytest
import torch

from loqa_hub_amd.config import GPUConfig
from loqa_hub_amd.engine.grammar import GrammarTables, multi_command_schema
from loqa_hub_amd.engine.tokenizer import HFTokenizer, find_tokenizer, load_tokenizer
from loqa_hub_amd.llm.commands import parse_multi_command_response
from loqa_hub_amd.llm.prompts import build_multi_command_prompt

tk = pytest.importorskip("tokenizers")

CORPUS = [build_multi_command_prompt(t) for t in (
    "turn on the kitchen lights and play music in the bedroom",
    "turn off the tv then dim the living room lamp",
    "hello what time is it 95 percent 0123456789")] * 20

WHISPER_SPECIALS = ["<|endoftext|>", "<|startoftranscript|>", "<|en|>", "<|transcribe|>",
                    "<|notimestamps|>", "<|de|>"]


def _byte_level(path, vocab=600, specials=("<|begin_of_text|>", "<|end_of_text|>")):
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers, trainers
    t = Tokenizer(models.BPE())
    t.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    t.decoder = decoders.ByteLevel()
    t.train_from_iterator(CORPUS, trainers.BpeTrainer(
        vocab_size=vocab, special_tokens=list(specials),
        initial_alphabet=pre_tokenizers.ByteLevel.alphabet()))
    os.makedirs(path, exist_ok=True)
    t.save(os.path.join(path, "tokenizer.json"))
    return os.path.join(path, "tokenizer.json")


def _metaspace(path, vocab=500):
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers, trainers
    t = Tokenizer(models.BPE(unk_token="<unk>"))
    t.pre_tokenizer = pre_tokenizers.Metaspace()
    t.decoder = decoders.Metaspace()
    alphabet = [chr(c) for c in range(32, 127)]
    t.train_from_iterator(CORPUS, trainers.BpeTrainer(vocab_size=vocab, initial_alphabet=alphabet,
                                                      special_tokens=["<unk>", "<s>", "</s>"]))
    os.makedirs(path, exist_ok=True)
    t.save(os.path.join(path, "tokenizer.json"))
    return os.path.join(path, "tokenizer.json")


@pytest.mark.parametrize("kind", ["byte_level", "metaspace"])
def test_hf_tokenizer_interface(tmp_path, kind):
    f = (_byte_level if kind == "byte_level" else _metaspace)(str(tmp_path / kind))
    tok = HFTokenizer(f, 4096)
    text = 'Voice command: "turn on the lights" {"confidence": 0.95}'
    ids = tok.encode(text, bos=True)
    assert ids[0] == tok.bos and tok.bos is not None and tok.eos is not None
    assert tok.decode(ids) == text
    # the texts the constrained decoder concatenates rebuild the input exactly
    # (a SentencePiece tokenizer adds its one leading space)
    joined = "".join(tok.token_text(t) for t in ids[1:])
    assert joined == (text if kind == "byte_level" else " " + text)
    for s in ['"', "0", "9", "{"]:
        assert tok.token_text(tok.token_id(s)) == s
    assert tok.token_text(tok.bos) == "" and tok.token_text(4095) == ""
    with pytest.raises(ValueError):
        HFTokenizer(f, 100)      # a file larger than the model's vocabulary


def test_find_tokenizer(tmp_path):
    f = _byte_level(str(tmp_path / "ckpt"))
    ckpt = tmp_path / "ckpt" / "model.safetensors"
    ckpt.write_bytes(b"")
    assert find_tokenizer(str(tmp_path / "ckpt")) == f
    assert find_tokenizer(str(ckpt)) == f
    assert find_tokenizer(f) == f
    assert find_tokenizer(str(tmp_path)) is None and find_tokenizer("") is None
    with pytest.raises(FileNotFoundError):
        load_tokenizer(str(tmp_path), 4096)
    g = GPUConfig(llm_checkpoint=str(ckpt))
    assert isinstance(g.tokenizer("llm", 4096), HFTokenizer)
    assert g.tokenizer("stt", 4096) is None            # no checkpoint: synthetic tokenizer
    g = GPUConfig(stt_tokenizer=f)
    assert isinstance(g.tokenizer("stt", 4096), HFTokenizer)


@pytest.mark.parametrize("kind", ["byte_level", "metaspace"])
def test_llm_engine_with_checkpoint_tokenizer_cpu(tmp_path, kind):
    """The constrained decoder on a real tokenizer: grammar tables from its
    vocabulary, prompts through its BPE, valid multi-command JSON out."""
    from loqa_hub_amd.engine.llm_engine import GenRequest, LLMEngine
    from loqa_hub_amd.models.configs import llama_config
    f = (_byte_level if kind == "byte_level" else _metaspace)(str(tmp_path / kind))
    tok = load_tokenizer(f, 4096)
    GrammarTables(tok)
    eng = LLMEngine(llama_config("test-tiny"), torch.device("cpu"), seed=0, max_seqs=4,
                    max_seq_len=768, use_graphs=False, tokenizer=tok)
    assert eng.tok is tok
    reqs = [GenRequest(tok.encode(build_multi_command_prompt("turn on the lights and play music"),
                                  bos=True), multi_command_schema(n)) for n in (1, 2)]
    eng.generate(reqs)
    for n, r in zip((1, 2), reqs):
        assert len(parse_multi_command_response(r.output, "x").commands) == n
        json.loads(r.output)


def test_stt_engine_with_checkpoint_tokenizer_cpu(tmp_path):
    """Whisper's special tokens come from the file; a teacher-forced
    transcript round-trips through the file's BPE."""
    from loqa_hub_amd.engine.stt_engine import STTEngine, STTRequest
    from loqa_hub_amd.engine.synthetic import make_batch
    from loqa_hub_amd.models.configs import whisper_config
    f = _byte_level(str(tmp_path / "whisper"), specials=WHISPER_SPECIALS)
    tok = load_tokenizer(f, 4096)
    eng = STTEngine(whisper_config("test-whisper"), torch.device("cpu"), seed=0, max_batch=4,
                    tokenizer=tok)
    assert eng.sot == [tok.token_id(s) for s in WHISPER_SPECIALS[1:5]]
    assert eng.eot == tok.token_id("<|endoftext|>") == 0
    utts = make_batch(0, 2, [1, 2])
    reqs = [STTRequest(u.pcm, transcript=u.text) for u in utts]
    eng.transcribe(reqs)
    for r, u in zip(reqs, utts):
        assert r.text == u.text
    # STT_LANGUAGE picks the language token of the start-of-transcript prompt
    de = STTEngine(whisper_config("test-whisper"), torch.device("cpu"), seed=0, max_batch=2,
                   tokenizer=tok, language="de", weights=eng.weights)
    assert de.sot[1] == tok.token_id("<|de|>") and de.sot[0] == eng.sot[0]
    with pytest.raises(ValueError):
        STTEngine(whisper_config("test-whisper"), torch.device("cpu"), seed=0, max_batch=2,
                  tokenizer=tok, language="fr", weights=eng.weights)


LLAMA3_TEMPLATE = (
    "{{ bos_token }}{% for m in messages %}<|start_header_id|>{{ m['role'] }}<|end_header_id|>\n\n"
    "{{ m['content'] | trim }}<|eot_id|>{% endfor %}"
    "{% if add_generation_prompt %}<|start_header_id|>assistant<|end_header_id|>\n\n{% endif %}")


def test_chat_template_prompt_cpu(tmp_path):
    """A checkpoint with a chat template gets its prompts wrapped as the user
    turn (as Ollama's /api/generate does for the reference); the decoder still
    emits valid multi-command JSON after the assistant header."""
    from loqa_hub_amd.engine.llm_engine import GenRequest, LLMEngine
    from loqa_hub_amd.models.configs import llama_config
    specials = ("<|begin_of_text|>", "<|end_of_text|>", "<|start_header_id|>", "<|end_header_id|>",
                "<|eot_id|>")
    f = _byte_level(str(tmp_path / "chat"), specials=specials)
    with open(tmp_path / "chat" / "tokenizer_config.json", "w") as fh:
        json.dump({"chat_template": LLAMA3_TEMPLATE, "bos_token": "<|begin_of_text|>",
                   "eos_token": {"content": "<|eot_id|>"}}, fh)
    tok = load_tokenizer(f, 4096)
    text = build_multi_command_prompt("turn on the lights")
    ids = tok.encode_prompt(text)
    hdr, end = tok.token_id("<|start_header_id|>"), tok.token_id("<|end_header_id|>")
    assert ids[0] == tok.bos and ids[1] == hdr and ids.count(hdr) == 2 and ids[-1] == tok.encode("\n\n")[-1]
    assert tok.decode(ids) == "user\n\n" + text.strip() + "assistant\n\n"
    assert end in ids and tok.token_id("<|eot_id|>") in ids
    # a tokenizer without a template: BOS + text
    plain = load_tokenizer(_byte_level(str(tmp_path / "plain")), 4096)
    assert plain.encode_prompt("hi") == [plain.bos] + plain.encode("hi")
    eng = LLMEngine(llama_config("test-tiny"), torch.device("cpu"), seed=0, max_seqs=2,
                    max_seq_len=768, use_graphs=False, tokenizer=tok)
    reqs = [GenRequest(ids, multi_command_schema(2))]
    eng.generate(reqs)
    assert len(parse_multi_command_response(reqs[0].output, "x").commands) == 2


def test_stt_suppression_with_checkpoint_tokenizer_cpu(tmp_path):
    """Greedy Whisper decoding on a checkpoint tokenizer never emits its
    special tokens (other than end-of-text) or the generation config's
    suppress_tokens; random weights would otherwise hit them."""
    from loqa_hub_amd.engine.stt_engine import STTEngine, STTRequest
    from loqa_hub_amd.engine.synthetic import make_batch
    from loqa_hub_amd.models.configs import whisper_config
    f = _byte_level(str(tmp_path / "whisper"), vocab=3000, specials=WHISPER_SPECIALS)
    suppressed = list(range(300, 2900))
    with open(tmp_path / "whisper" / "generation_config.json", "w") as fh:
        json.dump({"suppress_tokens": suppressed}, fh)
    tok = load_tokenizer(f, 4096)
    m = tok.sampling_mask(keep=(tok.token_id("<|endoftext|>"),))
    assert not m[300:2900].any() and not m[tok.n_real:].any() and m[0] and not m[1:6].any()
    eng = STTEngine(whisper_config("test-whisper"), torch.device("cpu"), seed=0, max_batch=4,
                    tokenizer=tok)
    utts = make_batch(0, 3, [1, 2])
    reqs = [STTRequest(u.pcm, max_new_tokens=12) for u in utts]
    eng.transcribe(reqs)
    allowed = set(m.nonzero().flatten().tolist())
    toks = [t for r in reqs for t in r.tokens]
    assert toks and set(toks) <= allowed


def test_byte_fallback_tokens_rank_after_pieces(tmp_path):
    """SentencePiece byte-fallback tokens (<0x22>, regular vocabulary entries
    ahead of the pieces, as in Llama-2 / TinyLlama files) decode to the same
    text as the real piece; token_id returns the piece (what a model emits)."""
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers
    vocab = {"<unk>": 0, "<s>": 1, "</s>": 2}
    for b in range(256):
        vocab[f"<0x{b:02X}>"] = len(vocab)
    for c in ["\u2581"] + [chr(c) for c in range(33, 127)]:
        vocab[c] = len(vocab)
    t = Tokenizer(models.BPE(vocab=vocab, merges=[], unk_token="<unk>", byte_fallback=True))
    t.pre_tokenizer = pre_tokenizers.Metaspace()
    t.decoder = decoders.Sequence([decoders.ByteFallback(), decoders.Metaspace()])
    t.add_special_tokens(["<unk>", "<s>", "</s>"])
    os.makedirs(tmp_path / "bf", exist_ok=True)
    t.save(str(tmp_path / "bf" / "tokenizer.json"))
    tok = HFTokenizer(str(tmp_path / "bf" / "tokenizer.json"), 4096)
    assert tok.token_text(vocab["<0x22>"]) == '"'             # same text as the piece
    assert tok.token_id('"') == vocab['"'] and tok.token_id("0") == vocab["0"]


def test_hub_processor_uses_checkpoint_and_tokenizer_cpu(tmp_path):
    """HUB_LLM_CHECKPOINT pointing at a safetensors directory with a
    tokenizer.json: the served processor's engine loads both, and an
    utterance runs through the hub path on them."""
    import asyncio

    import numpy as np

    from loqa_hub_amd import config as cfgmod
    from loqa_hub_amd.models import loader
    from loqa_hub_amd.models.configs import llama_config
    from loqa_hub_amd.models.llama import LlamaWeights
    from loqa_hub_amd.server import build_gpu_processor
    ck = tmp_path / "llm"
    os.makedirs(ck)
    w = LlamaWeights(llama_config("test-tiny"), torch.device("cpu"), seed=5)
    loader.save_llama(w, str(ck / "model.safetensors"))
    _byte_level(str(ck))
    with open(ck / "config.json", "w") as fh:     # the shape comes from the checkpoint
        json.dump({"hidden_size": 256, "num_hidden_layers": 2, "num_attention_heads": 4,
                   "num_key_value_heads": 2, "intermediate_size": 512, "vocab_size": 4096,
                   "tie_word_embeddings": True, "max_position_embeddings": 2048}, fh)

    async def go():
        cfg = cfgmod.load({"HUB_STT_MODEL": "test-whisper", "HUB_LLM_MODEL": "llama3-8b",
                           "HUB_MAX_BATCH": "2", "HUB_USE_GRAPHS": "false",
                           "HUB_LLM_CHECKPOINT": str(ck), "HUB_TTS_BACKEND": "none"})
        proc = build_gpu_processor(cfg, None, device="cpu", bridge=False)
        eng = proc.pipeline.llm
        assert eng.cfg.d_model == 256 and eng.cfg.n_layers == 2   # not the named llama3-8b
        assert isinstance(eng.tok, HFTokenizer)
        assert torch.equal(eng.weights.layers[0]["wqkv"].float(), w.layers[0]["wqkv"].float())
        pcm = np.random.default_rng(0).standard_normal(16000).astype(np.float32) * 0.1
        r = await proc.process("r0", "q0", pcm, 16000)
        assert r.command in ("voice_command_success", "no_speech", "error", "confirmation_needed")
    asyncio.run(go())
