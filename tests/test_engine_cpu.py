"""Engine-level CPU tests: tokenizer, grammar-constrained decoding, paged-KV block
pools (Python and native C++), torch references of the HIP ops, the LLM / STT
engines on tiny configs, the voice pipeline, and the DP bench path over gloo."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from loqa_hub_amd.engine.grammar import (Choice, Digits, Free, GrammarState, GrammarTables, Lit,
                                         multi_command_schema, single_command_schema)
from loqa_hub_amd.engine.kv_cache import PyBlockPool
from loqa_hub_amd.engine.tokenizer import get_tokenizer
from loqa_hub_amd.llm.commands import parse_multi_command_response, parse_response
from loqa_hub_amd.ops import reference as R

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_tokenizer_roundtrip():
    tok = get_tokenizer(32000)
    for s in ['{"intent": "turn_on"}', "turn on the kitchen lights, then play music",
              "émoji ✓ bytes"]:
        ids = tok.encode(s)
        assert tok.decode(ids) == s
        assert all(0 <= i < tok.vocab_size for i in ids)
    assert tok.vocab_size == 32000


def _walk(state: GrammarState, tables: GrammarTables, rng) -> str:
    state.start()
    for _ in range(2000):
        row = state.mask_row()
        if row < 0:
            break
        allowed = tables.allowed(row).nonzero().flatten().tolist()
        state.advance(int(rng.choice(allowed)))
    assert state.done
    return state.text()


@pytest.mark.parametrize("n", [1, 2, 3])
def test_grammar_random_walk_is_valid_json(n):
    tok = get_tokenizer(32000)
    tables = GrammarTables(tok)
    rng = np.random.default_rng(n)
    for trial in range(5):
        text = _walk(GrammarState(tables, multi_command_schema(n)), tables, rng)
        obj = json.loads(text)
        assert len(obj["commands"]) == n
        mc = parse_multi_command_response(text, "x")
        assert all(c.intent in ("turn_on", "turn_off", "greeting", "question", "unknown")
                   for c in mc.commands)
    single = _walk(GrammarState(tables, single_command_schema()), tables, rng)
    assert parse_response(single).intent


def test_grammar_min_length_and_digits():
    tok = get_tokenizer(32000)
    tables = GrammarTables(tok)
    st = GrammarState(tables, [Lit('{"a": "'), Free("a", 4, min_tokens=2), Lit('", "d": 0.'),
                               Digits(2), Lit("}")])
    st.start()
    assert st.mask_row() == tables.ROW_FREE_OPEN  # quote not allowed yet
    assert not bool(tables.allowed(st.mask_row())[tables.quote])
    st.advance(tok.token_id("x"))
    st.advance(tok.token_id("y"))
    assert st.mask_row() == tables.ROW_FREE
    st.advance(tables.quote)
    # two digits in one token (Llama-3 BPE keeps numbers <= 999 whole)
    assert st.mask_row() == tables.ROW_DIGIT2
    assert bool(tables.allowed(st.mask_row())[tok.token_id("42")])
    assert not bool(tables.allowed(st.mask_row())[tok.token_id("4")])
    st.advance(tok.token_id("42"))
    assert st.done and json.loads(st.text()) == {"a": "xy", "d": 0.42}
    # a single-digit field still samples from the one-digit row
    st = GrammarState(tables, [Lit("0."), Digits(1)])
    st.start()
    assert st.mask_row() == tables.ROW_DIGIT
    st.advance(tok.token_id("7"))
    assert st.done and st.text() == "0.7"
    # choice trie: forced completion once the prefix is unique
    st = GrammarState(tables, [Lit('"'), Choice("c", ["turn_on", "turn_off"]), Lit('"')])
    st.start()
    while not st.done:
        st.advance(int(tables.allowed(st.mask_row()).nonzero()[0]))
    assert json.loads(st.text()) in ("turn_on", "turn_off")


def test_mask_pack_roundtrip():
    m = torch.rand(3, 100) > 0.5
    packed = R.pack_mask(m)
    assert packed.dtype == torch.int32 and packed.shape == (3, 4)
    assert torch.equal(R.unpack_mask(packed, 100), m)


def _exercise_pool(pool):
    toks = list(range(40))
    assert pool.add_seq(1, toks) == 0
    slots = pool.append(1, 40)
    assert len(slots) == 40 and len(set(slots)) == 40
    assert pool.seq_len(1) == 40 and len(pool.block_table(1)) == 3
    pool.cache_prefix(1, toks)
    hit = pool.add_seq(2, toks[:32] + [99, 98])
    assert hit == 32  # two full blocks shared
    assert pool.block_table(2)[:2] == pool.block_table(1)[:2]
    before = pool.free_blocks()
    pool.append(2, 20)
    assert pool.seq_len(2) == 52 and pool.free_blocks() < before
    pool.free_seq(1)
    pool.free_seq(2)
    assert pool.add_seq(3, toks[:16] + [7]) == 16  # cached block survives until evicted
    pool.free_seq(3)
    # exhausting the pool evicts unreferenced cached blocks instead of failing
    assert pool.add_seq(4, [5]) == 0
    assert pool.append(4, 16 * pool_blocks(pool)) is not None


def pool_blocks(pool):
    return 64


def test_py_block_pool():
    _exercise_pool(PyBlockPool(64, 16))


def test_native_block_pool_matches():
    from loqa_hub_amd.engine.kv_cache import NativeBlockPool
    from loqa_hub_amd.ops import _lib
    try:
        _lib.runtime()
    except Exception as e:  # noqa: BLE001
        pytest.skip(f"native runtime not built: {e}")
    _exercise_pool(NativeBlockPool(64, 16))


def test_native_prefix_cache_survives_hash_collisions():
    """Every prefix hash forced to collide: hits must still be decided by the
    stored tokens (a collision must never reuse another prompt's KV)."""
    from loqa_hub_amd.engine.kv_cache import NativeBlockPool
    from loqa_hub_amd.ops import _lib
    try:
        _lib.runtime()
    except Exception as e:  # noqa: BLE001
        pytest.skip(f"native runtime not built: {e}")
    pool = NativeBlockPool(64, 16)
    pool.lib.loqa_pool_debug_hash_mask(pool.h, 0)
    a = list(range(48))
    b = list(range(100, 148))
    for sid, toks in ((1, a), (2, b)):
        assert pool.add_seq(sid, toks) == 0
        pool.append(sid, len(toks))
        pool.cache_prefix(sid, toks)
    # same hash for every block of a and b: only exact token prefixes hit
    assert pool.add_seq(3, b[:32] + [1]) == 32
    assert pool.block_table(3)[:2] == pool.block_table(2)[:2]
    assert pool.add_seq(4, a[:16] + b[16:32] + [1]) == 16     # block 2 differs -> stops
    assert pool.block_table(4)[:1] == pool.block_table(1)[:1]
    assert pool.add_seq(5, [7] * 40) == 0
    for sid in range(1, 6):
        pool.free_seq(sid)
    # cached blocks are evicted (not leaked) when the pool runs dry
    assert pool.add_seq(6, [5]) == 0
    assert pool.append(6, 16 * 64) is not None


def test_skinny_reference_and_shuffle():
    torch.manual_seed(0)
    N, K = 64, 256
    W = torch.randn(N, K).bfloat16()
    Wp = R.shuffle_weight(W)
    assert torch.equal(R.unshuffle_weight(Wp), W)
    x = torch.randn(16, K).bfloat16()
    part = R.skinny_gemm(x, Wp, 4)
    assert part.shape == (4, 16, N)
    assert torch.allclose(part.sum(0), x.float() @ W.float().t(), atol=1e-3, rtol=1e-4)


def test_attention_reference_matches_sdpa():
    torch.manual_seed(0)
    q = torch.randn(2, 4, 10, 64)
    k = torch.randn(2, 2, 10, 64)
    v = torch.randn(2, 2, 10, 64)
    kk, vv = k.repeat_interleave(2, 1), v.repeat_interleave(2, 1)
    ref = torch.nn.functional.scaled_dot_product_attention(q, kk, vv, is_causal=True)
    s = (q @ kk.transpose(-1, -2)) / 8.0
    s = s.masked_fill(torch.ones(10, 10, dtype=torch.bool).triu(1), float("-inf"))
    assert torch.allclose(s.softmax(-1) @ vv, ref, atol=1e-5)


def test_llm_engine_cpu_generates_valid_json():
    from loqa_hub_amd.engine.llm_engine import GenRequest, LLMEngine
    from loqa_hub_amd.models.configs import llama_config
    eng = LLMEngine(llama_config("test-tiny"), torch.device("cpu"), seed=0, max_seqs=4,
                    max_seq_len=512, use_graphs=False)
    reqs = [GenRequest(eng.tok.encode("turn on the lights and play music", bos=True),
                       multi_command_schema(n)) for n in (1, 2, 3)]
    eng.generate(reqs)
    for n, r in zip((1, 2, 3), reqs):
        mc = parse_multi_command_response(r.output, "x")
        assert len(mc.commands) == n
    assert eng.stats["decode_steps"] > 0


def test_stt_engine_cpu_teacher_forced():
    from loqa_hub_amd.engine.stt_engine import STTEngine, STTRequest
    from loqa_hub_amd.engine.synthetic import make_batch
    from loqa_hub_amd.models.configs import whisper_config
    eng = STTEngine(whisper_config("test-whisper"), torch.device("cpu"), seed=0, max_batch=4)
    utts = make_batch(0, 3, [1, 2])
    reqs = [STTRequest(u.pcm, transcript=u.text) for u in utts]
    eng.transcribe(reqs)
    for r, u in zip(reqs, utts):
        assert r.text == u.text


def _run(cmd, timeout=600):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="2")
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_cpu_smoke_single():
    out = _run([sys.executable, "bench.py", "--cpu-smoke", "--steps", "1", "--warmup", "0",
                "--batch-per-gpu", "4"])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in out
    assert out["n_gpus"] == 1 and out["queue_success_rate"] == 1.0
    assert out["command_count_match_rate"] == 1.0


def test_bench_cpu_smoke_dp2_gloo():
    out = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node",
                "2", "--master-addr", "127.0.0.1", "--master-port", "29561", "bench.py",
                "--cpu-smoke", "--gpus", "2", "--steps", "1", "--warmup", "0",
                "--batch-per-gpu", "2"])
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2"
    assert out["config"]["global_batch"] == 4 and out["queue_success_rate"] == 1.0


def test_bench_cpu_smoke_dp4_gloo():
    """Four ranks (the driver runs 1/2/4/8): one NATS broker process for the
    node, every rank publishes to it, records are all-gathered to rank 0."""
    out = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node",
                "4", "--master-addr", "127.0.0.1", "--master-port", "29563", "bench.py",
                "--cpu-smoke", "--gpus", "4", "--steps", "1", "--warmup", "0",
                "--batch-per-gpu", "2"])
    assert out["n_gpus"] == 4 and out["config"]["parallelism"] == "dp4"
    assert out["config"]["global_batch"] == 8 and out["queue_success_rate"] == 1.0
    assert out["command_count_match_rate"] == 1.0


def test_bench_cpu_smoke_dp8_gloo():
    """Eight ranks - the width the driver launches on an 8-GPU node
    (torchrun --nproc-per-node 8): per-rank served hubs (the default hub mode,
    gRPC relays), one NATS broker, records gathered to rank 0."""
    out = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node",
                "8", "--master-addr", "127.0.0.1", "--master-port", "29565", "bench.py",
                "--cpu-smoke", "--gpus", "8", "--steps", "1", "--warmup", "0",
                "--batch-per-gpu", "1", "--window-steps", "0"], timeout=900)
    assert out["n_gpus"] == 8 and out["config"]["parallelism"] == "dp8"
    assert out["config"]["mode"] == "hub" and out["config"]["global_batch"] == 8
    assert out["queue_success_rate"] == 1.0 and out["command_count_match_rate"] == 1.0


def test_bench_rank_without_device_fails_fast(monkeypatch):
    """A GPU run whose rank has no device of its own exits 2 with a message
    before any collective."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    args = type("A", (), {"cpu_smoke": False, "gpus": 8})()
    monkeypatch.setattr(bench.torch.cuda, "device_count", lambda: 4)
    monkeypatch.setenv("LOCAL_RANK", "5")
    monkeypatch.setenv("RANK", "5")
    monkeypatch.delenv("LOQA_DIST_SHARE_GPU", raising=False)
    assert "has no GPU" in bench.rank_device_problem(args)
    monkeypatch.setenv("LOCAL_RANK", "3")
    assert bench.rank_device_problem(args) is None
    monkeypatch.setattr(bench.torch.cuda, "device_count", lambda: 0)
    assert "no GPU visible" in bench.rank_device_problem(args)
    args.cpu_smoke = True
    assert bench.rank_device_problem(args) is None


def test_bench_gpus_guard():
    """--gpus must match the launch: a torchrun job of the wrong size exits 2;
    without torchrun, --gpus 2 relaunches the bench under torch.distributed.run."""
    import subprocess
    env = dict(os.environ, WORLD_SIZE="1")
    r = subprocess.run([sys.executable, "bench.py", "--cpu-smoke", "--gpus", "2", "--steps", "1"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 2 and "WORLD_SIZE" in r.stderr
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "bench.py", "--cpu-smoke", "--gpus", "2", "--steps", "1",
                        "--warmup", "0", "--batch-per-gpu", "2"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2"


def test_bench_cpu_smoke_hub_mode():
    """--mode hub: relays over gRPC into the served hub (arbitration, bridge,
    voice events) on the same pipeline."""
    out = _run([sys.executable, "bench.py", "--cpu-smoke", "--steps", "1",
                "--warmup", "1", "--batch-per-gpu", "2", "--window-ms", "10",
                "--window-steps", "1"])
    # hub mode + single-relay bypass are the defaults; the window_300ms pass
    # (bypass off) adds one utterance per relay after the timed step
    assert out["config"]["mode"] == "hub" and out["queue_success_rate"] == 1.0
    # one voice event per timed utterance (the warm-up step's are counted apart)
    hub = out["hub"]
    assert hub["voice_events"] == 2 == hub["timed_utterances"] and hub["voice_events_total"] == 4
    svc = hub["audio_service"]
    assert svc["processed"] == 4 and svc["bypassed"] == 4
    w = out["window_300ms"]
    assert w["utterances"] == 2 and w["utterances_per_sec"] > 0 and w["window_ms"] == 10


def test_whisper_fast_decode_matches_eager_cpu():
    """The skinny-GEMM/slab decode path equals the eager reference decoder
    (first step with the 4 SOT tokens and a follow-up 1-token step)."""
    from loqa_hub_amd.engine.stt_engine import STTEngine, STTRequest
    from loqa_hub_amd.engine.synthetic import make_batch
    from loqa_hub_amd.models.configs import whisper_config
    cfg = whisper_config("test-whisper")
    utts = make_batch(1, 2, [1, 2])
    modes = ("fused", "fast", "eager")
    engines = [STTEngine(cfg, torch.device("cpu"), seed=3, max_batch=4, fast_decode=m != "eager")
               for m in modes]
    outs = []
    for mode, eng in zip(modes, engines):
        reqs = [STTRequest(u.pcm) for u in utts]
        audio, _ = eng.upload(reqs)
        eng.cross_kv(eng.model.encode(audio))
        for i, r in enumerate(reqs):
            r.seq_id = eng._next
            r.slot = i
            r.feed = list(eng.sot)
            eng._next += 1
            eng.kv.pool.add_seq(r.seq_id, [])
        B_pad, T_pad = 2, 16
        res = []
        for step in range(2):
            max_q, host = eng._host_meta(reqs, B_pad, T_pad)
            dev = eng._dev(host)
            if mode == "fused":
                from loqa_hub_amd.models.whisper import decode_step_fused
                lg = decode_step_fused(eng.model, dev["tokens"], dev["positions"], dev["slots"],
                                       dev["cu_q"], dev["ctx_lens"], dev["block_tables"], max_q,
                                       eng.kv.k, eng.kv.v, eng.xkv, dev["enc_starts"],
                                       dev["enc_lens"], dev["logit_idx"], eng.ws, eng.scratch,
                                       eng.self_splits)
                lg = lg[:2, : cfg.vocab_size].float()
            elif mode == "fast":
                from loqa_hub_amd.models.whisper import decode_step_fast
                lg = decode_step_fast(eng.model, dev["tokens"], dev["positions"], dev["slots"],
                                      dev["cu_q"], dev["ctx_lens"], dev["block_tables"], max_q,
                                      eng.kv.k, eng.kv.v, eng.xkv, dev["enc_starts"],
                                      dev["enc_lens"], dev["logit_idx"], eng.ws, eng.self_splits)
                lg = lg[:2, : cfg.vocab_size].float()
            else:
                T = int(host["cu_q"][2])
                lg = eng.model.decode_step(
                    dev["tokens"][:T], dev["positions"][:T], dev["slots"][:T], dev["cu_q"][:3],
                    dev["ctx_lens"][:2], dev["block_tables"][:2], max_q, int(host["ctx_lens"].max()),
                    eng.kv.k, eng.kv.v, eng.xkv, dev["enc_starts"][:2], dev["enc_lens"][:2],
                    dev["logit_idx"][:2], None).float()
            res.append(lg)
            reqs[0].feed, reqs[1].feed = [11], [12]
        outs.append(res)
    for other in outs[:2]:
        for a, b in zip(other, outs[2]):
            err = (a - b).abs().max().item()
            assert err <= 2e-2 * b.abs().max().item() + 1e-3, err


def test_vits_tts_cpu():
    import asyncio
    from loqa_hub_amd.engine.tts_engine import VitsTTSEngine, wav_info
    from loqa_hub_amd.llm.tts import TTSOptions
    from loqa_hub_amd.models.configs import VITS_CONFIGS
    e = VitsTTSEngine(VITS_CONFIGS["test-vits"], "cpu")
    outs = e.synthesize_batch(["Turning on the lights.", "Hi!"])
    assert outs[0].size % 256 == 0 and outs[0].size > outs[1].size
    assert np.abs(outs[0].astype(np.float32)).mean() > 100

    async def go():
        r1, r2 = await asyncio.gather(e.synthesize("hello"), e.synthesize("world", TTSOptions(
            speed=2.0, response_format="pcm")))
        assert r1.content_type == "audio/wav" and wav_info(r1.audio)[0] == 22050
        assert r2.content_type == "audio/pcm" and len(r2.audio) % 2 == 0
    asyncio.run(go())
    assert e.stats["batches"] >= 2


def test_vits_tts_response_format_cpu():
    """response_format (openai_tts_client.go:39-46): wav / pcm as asked; a
    format the GPU voice cannot encode (the status manager's mp3,
    status_manager.go:441-462) is a counted, logged downgrade to WAV labelled
    "wav" by default, an error under format_policy="error"."""
    import asyncio
    import pytest as _pt
    from loqa_hub_amd.engine.tts_engine import UnsupportedAudioFormat, VitsTTSEngine, wav_info
    from loqa_hub_amd.llm.tts import TTSOptions
    from loqa_hub_amd.models.configs import VITS_CONFIGS
    e = VitsTTSEngine(VITS_CONFIGS["test-vits"], "cpu")

    async def go():
        w, p, m, o = await asyncio.gather(
            e.synthesize("hello", TTSOptions(response_format="wav")),
            e.synthesize("hello", TTSOptions(response_format="pcm")),
            e.synthesize("hello", TTSOptions("af_bella", 1.1, "mp3", True)),
            e.synthesize("hello", TTSOptions(response_format="opus")))
        assert (w.format, w.content_type) == ("wav", "audio/wav") and wav_info(w.audio)[0] == 22050
        assert (p.format, p.content_type) == ("pcm", "audio/pcm")
        for r in (m, o):   # never mp3 / opus bytes under a wav label or vice versa
            assert (r.format, r.content_type) == ("wav", "audio/wav") and r.audio[:4] == b"RIFF"
    asyncio.run(go())
    assert e.stats["format_downgrades"] == 2
    strict = VitsTTSEngine(VITS_CONFIGS["test-vits"], "cpu", format_policy="error")
    with _pt.raises(UnsupportedAudioFormat):
        asyncio.run(strict.synthesize("hello", TTSOptions(response_format="mp3")))
    assert asyncio.run(strict.synthesize("hi", TTSOptions(response_format="PCM"))).format == "pcm"
    with _pt.raises(ValueError):
        VitsTTSEngine(VITS_CONFIGS["test-vits"], "cpu", format_policy="mp3")


def test_vits_padding_is_inert_cpu():
    """The graph runner's buckets pad symbols, batch rows and frames: a row
    inside a padded batch (longer symbol axis, an extra row, frames rounded
    up) gets exactly the text statistics, durations, prior sample and
    reverse-flow latent it gets alone. (The vocoder's CPU convolutions pick
    batch-size-dependent algorithms, so its bitwise check runs on the GPU:
    tests/test_engine_gpu.py::test_vits_graph_runner_matches_eager_gpu.)"""
    from loqa_hub_amd import ops
    from loqa_hub_amd.models.configs import VITS_CONFIGS
    from loqa_hub_amd.models.vits import VitsModel, VitsWeights, text_to_ids
    cfg = VITS_CONFIGS["test-vits"]
    m = VitsModel(VitsWeights(cfg, "cpu", seed=2))
    a, b = text_to_ids("Lights on.", cfg.n_symbols), text_to_ids("Done", cfg.n_symbols)
    with torch.inference_mode():
        s1, c1, f1 = m.text_phase(torch.tensor([a]), torch.tensor([len(a)], dtype=torch.int32), 1.0)
        T = len(a) + 9
        ids = torch.zeros(2, T, dtype=torch.int64)
        ids[0, :len(a)] = torch.tensor(a)
        ids[1, :len(b)] = torch.tensor(b)
        s2, c2, f2 = m.text_phase(ids, torch.tensor([len(a), len(b)], dtype=torch.int32), 1.0)
        assert torch.equal(s2[0, :len(a)], s1[0]) and torch.equal(c2[0, :len(a)], c1[0])
        assert int(f2[0]) == int(f1[0])
        F = -(-int(f1[0]) // 64) * 64
        z1 = m.flow_reverse(ops.expand_sample(s1, c1, f1, F, 0.667, 4), f1)
        z2 = m.flow_reverse(ops.expand_sample(s2, c2, f2, F, 0.667, 4), f2)
        assert torch.equal(z1[0], z2[0]) and not z1[0, int(f1[0]):].any()
        pcm, n = m.synthesize(ids, torch.tensor([len(a), len(b)], dtype=torch.int32), seed=4,
                              frame_step=64)
    assert pcm.shape[1] % (64 * m.hop) == 0 and int(n[0]) == int(f1[0]) * m.hop


def test_conv_transpose_polyphase_cpu():
    from loqa_hub_amd import ops
    torch.manual_seed(0)
    for Cin, Cout, K, s in ((64, 32, 16, 8), (32, 32, 4, 2)):
        p = (K - s) // 2
        w, b = torch.randn(Cin, Cout, K) * 0.1, torch.randn(Cout) * 0.1
        x = torch.randn(2, 13, Cin).bfloat16()
        ct = ops.ConvTransposeWeight(w, b, s, p)
        y1 = ops.conv_transpose1d(x, ct, pre_slope=0.1, polyphase=True).float()
        y2 = R.conv_transpose1d(x, w, b, stride=s, padding=p, pre_slope=0.1)
        assert y1.shape == y2.shape and (y1 - y2).abs().max() <= 0.02 * y2.abs().max()


def test_llm_continuous_batching_scheduler_cpu():
    """Requests submitted while others decode join the running batch; every
    request completes with its schema's command count and KV blocks are freed."""
    import time as _t

    from loqa_hub_amd.engine.llm_engine import GenRequest, LLMEngine
    from loqa_hub_amd.models.configs import llama_config
    eng = LLMEngine(llama_config("test-tiny"), torch.device("cpu"), seed=0, max_seqs=8,
                    max_seq_len=512, use_graphs=False)
    free0 = eng.kv.pool.free_blocks()
    mk = lambda ns: [GenRequest(eng.tok.encode(f"turn on the lights {n}", bos=True),
                                multi_command_schema(n, min_response_tokens=2)) for n in ns]
    seen = []
    a = eng.submit_batch(mk((1, 3)), on_done=lambda r: seen.append(r.seq_id))
    _t.sleep(0.05)
    b = eng.submit_batch(mk((2, 4)))
    ra, rb = a.result(timeout=120), b.result(timeout=120)
    for n, r in zip((1, 3, 2, 4), ra + rb):
        assert len(parse_multi_command_response(r.output, "x").commands) == n
    assert sorted(seen) == sorted(r.seq_id for r in ra)
    eng.stop()
    assert eng.kv.pool.free_blocks() == free0


def test_pipeline_submit_continuous_cpu():
    import asyncio

    from loqa_hub_amd.engine.llm_engine import LLMEngine
    from loqa_hub_amd.engine.pipeline import PipelineJob, VoicePipeline
    from loqa_hub_amd.engine.stt_engine import STTEngine
    from loqa_hub_amd.engine.synthetic import make_batch
    from loqa_hub_amd.models.configs import llama_config, whisper_config
    stt = STTEngine(whisper_config("test-whisper"), torch.device("cpu"), seed=0, max_batch=4)
    llm = LLMEngine(llama_config("test-tiny"), torch.device("cpu"), seed=0, max_seqs=8,
                    max_seq_len=1024, use_graphs=False)
    pipe = VoicePipeline(stt, llm, None, min_response_tokens=2, continuous=True, max_batch=4)
    utts = make_batch(1, 4, [1, 2, 3, 4])

    async def go():
        async def one(i, u, delay):
            await asyncio.sleep(delay)
            return await pipe.submit(PipelineJob(u.relay_id, f"r{i}", u.pcm, transcript_hint=u.text))
        return await asyncio.gather(*[one(i, u, 0.03 * i) for i, u in enumerate(utts)])
    jobs = asyncio.run(go())
    llm.stop()
    assert [j.n_commands for j in jobs] == [j.n_expected for j in jobs] == [1, 2, 3, 4]
    assert pipe.stats["utterances"] == 4


def test_stt_continuous_batching_matches_batch_cpu():
    """Requests that join a RUNNING Whisper decode batch (scheduler thread,
    per-request cross-attention slots) decode exactly as in a one-shot batch."""
    import time as _t

    from loqa_hub_amd.engine.stt_engine import STTEngine, STTRequest
    from loqa_hub_amd.engine.synthetic import make_batch
    from loqa_hub_amd.models.configs import whisper_config
    cfg = whisper_config("test-whisper")
    utts = make_batch(5, 4, [1, 2, 3, 1])
    ref = STTEngine(cfg, torch.device("cpu"), seed=2, max_batch=4)
    solo = [STTRequest(u.pcm, max_new_tokens=6) for u in utts]
    ref.transcribe(solo)
    eng = STTEngine(cfg, torch.device("cpu"), seed=2, max_batch=4)
    a = [STTRequest(u.pcm, max_new_tokens=6) for u in utts[:2]]
    b = [STTRequest(u.pcm, max_new_tokens=6) for u in utts[2:3]]
    c = [STTRequest(u.pcm, transcript=u.text) for u in utts[3:]]
    seen = []
    fa = eng.submit_batch(a, lambda r: seen.append(r))
    _t.sleep(0.05)                      # b and c arrive mid-decode
    fb = eng.submit_batch(b)
    fc = eng.submit_batch(c)
    for f in (fa, fb, fc):
        f.result(timeout=120)
    eng.stop()
    assert len(seen) == 2
    for got, want in zip(a + b, solo[:3]):
        assert got.tokens == want.tokens
        assert abs(got.rms - want.rms) < 1e-6
    assert c[0].text.lower().startswith(utts[3].text.lower().split()[0])
    assert sorted(eng._free_slots) == list(range(4))


def test_stt_oversize_batch_is_chunked_cpu():
    """A batch larger than the engine's slot count is admitted in max_batch
    chunks (it would otherwise never find enough free slots)."""
    from loqa_hub_amd.engine.stt_engine import STTEngine, STTRequest
    from loqa_hub_amd.engine.synthetic import make_batch
    from loqa_hub_amd.models.configs import whisper_config
    cfg = whisper_config("test-whisper")
    utts = make_batch(7, 5, [1, 2, 1, 1, 2])
    ref = STTEngine(cfg, torch.device("cpu"), seed=2, max_batch=8)
    solo = [STTRequest(u.pcm, max_new_tokens=4) for u in utts]
    ref.transcribe(solo)
    eng = STTEngine(cfg, torch.device("cpu"), seed=2, max_batch=2)
    reqs = [STTRequest(u.pcm, max_new_tokens=4) for u in utts]
    done = []
    out = eng.submit_batch(reqs, lambda r: done.append(r)).result(timeout=120)
    eng.stop()
    assert out == reqs and len(done) == 5
    for got, want in zip(reqs, solo):
        assert got.tokens == want.tokens
    assert sorted(eng._free_slots) == [0, 1]


def test_pipeline_continuous_stt_cpu():
    """Pipeline with continuous STT + continuous LLM on the CPU: every utterance
    gets its own reply with the expected command count."""
    import asyncio

    from loqa_hub_amd.engine.llm_engine import LLMEngine
    from loqa_hub_amd.engine.pipeline import PipelineJob, VoicePipeline
    from loqa_hub_amd.engine.stt_engine import STTEngine
    from loqa_hub_amd.engine.synthetic import make_batch
    from loqa_hub_amd.models.configs import llama_config, whisper_config
    stt = STTEngine(whisper_config("test-whisper"), torch.device("cpu"), seed=0, max_batch=4)
    llm = LLMEngine(llama_config("test-tiny"), torch.device("cpu"), seed=0, max_seqs=8,
                    max_seq_len=1024, use_graphs=False)
    pipe = VoicePipeline(stt, llm, None, min_response_tokens=2, continuous=True,
                         stt_continuous=True, max_batch=4)
    utts = make_batch(1, 6, [1, 2, 3])

    async def main():
        jobs = [PipelineJob(u.relay_id, f"r{i}", u.pcm, transcript_hint=u.text)
                for i, u in enumerate(utts)]
        return await asyncio.gather(*[pipe.submit(j) for j in jobs])
    try:
        res = asyncio.run(main())
    finally:
        stt.stop()
        llm.stop()
    assert [j.n_commands for j in res] == [u.n_commands for u in utts]
    assert all(j.queue is not None and j.transcription is not None for j in res)


def test_llm_compact_weights_match_default_cpu():
    """Compact single-copy weights (fused layout only, chunked fused prefill)
    compute the same model as the default two-copy layout: the logits of the
    prompt's last position agree (the paths round to bf16 at different points,
    so a sampled near-tie may flip later on), and the constrained outputs are
    valid with the same structure."""
    import json

    from loqa_hub_amd.engine.grammar import multi_command_schema
    from loqa_hub_amd.engine.llm_engine import GenRequest, LLMEngine
    from loqa_hub_amd.models.configs import llama_config
    cfg = llama_config("test-tiny")
    outs, logits = [], []
    prompt = list(range(10, 10 + 70))
    for compact in (False, True):
        eng = LLMEngine(cfg, torch.device("cpu"), seed=4, max_seqs=4, max_seq_len=512,
                        use_graphs=False, compact=compact)
        if compact:
            assert "wqkv" not in eng.weights.layers[0] and "wqkv_f" in eng.weights.decode_layers[0]
        r = GenRequest(prompt, [])
        r.seq_id = eng._next_id
        eng._next_id += 1
        eng.kv.pool.add_seq(r.seq_id, [])
        if compact:      # 64-token chunks through the fused decode step
            for c0 in range(0, len(prompt), 64):
                chunk = prompt[c0:c0 + 64]
                max_q, max_ctx, host = eng._meta([r], [chunk], True, 1, 128 if len(chunk) > 64 else 64)
                meta = eng._build_meta(eng._to_device(host), max_q, max_ctx, True)
                lg = eng.model.forward_decode_fused(meta, eng.kv.k, eng.kv.v, eng.attn_ws,
                                                    eng.scratch)[:1]
        else:
            max_q, max_ctx, host = eng._meta([r], [prompt], decode=False)
            meta = eng._build_meta(eng._to_device(host), max_q, max_ctx, False)
            lg = eng.model.logits(eng.model.forward(meta, eng.kv.k, eng.kv.v, eng.attn_ws))
        eng.kv.pool.free_seq(r.seq_id)
        logits.append(lg.float())
        reqs = [GenRequest(list(range(10, 10 + 70 + 9 * i)), multi_command_schema(2, min_response_tokens=2))
                for i in range(2)]
        eng.generate(reqs)
        outs.append([json.loads(r.output) for r in reqs])
    err = (logits[0] - logits[1]).abs().max().item()
    assert err <= 0.02 * logits[0].abs().max().item(), err
    for a, b in zip(*outs):
        assert len(a["commands"]) == len(b["commands"]) == 2


def test_llm_compact_weights_scheduler_cpu():
    """compact weights keep no row-major prompt-pass copies, so the
    continuous-batching scheduler must not send their prompts (> 64 tokens,
    the default inline limit) into a mixed pass (model.forward -> KeyError);
    they go through the fused chunked prefill and produce the same outputs
    as generate()."""
    import json

    from loqa_hub_amd.engine.grammar import multi_command_schema
    from loqa_hub_amd.engine.llm_engine import GenRequest, LLMEngine
    from loqa_hub_amd.models.configs import llama_config
    cfg = llama_config("test-tiny")
    eng = LLMEngine(cfg, torch.device("cpu"), seed=4, max_seqs=4, max_seq_len=512,
                    use_graphs=False, compact=True)

    def reqs():
        return [GenRequest(list(range(10, 10 + 90 + 9 * i)),
                           multi_command_schema(1 + i, min_response_tokens=2)) for i in range(3)]
    ref = [r.output for r in eng.generate(reqs())]
    try:
        got = eng.submit_batch(reqs()).result(timeout=120)
    finally:
        eng.stop()
    assert [r.output for r in got] == ref
    assert [len(json.loads(o)["commands"]) for o in ref] == [1, 2, 3]


def test_step_meta_native_matches_python():
    """One-call step metadata (native) against the Python twin."""
    from loqa_hub_amd.engine.kv_cache import NativeBlockPool
    from loqa_hub_amd.ops import _lib
    try:
        _lib.runtime()
    except Exception as e:  # noqa: BLE001
        pytest.skip(f"native runtime not built: {e}")
    rng = np.random.default_rng(0)
    pools = [PyBlockPool(128, 16), NativeBlockPool(128, 16)]
    for p in pools:
        for sid in range(1, 6):
            assert p.add_seq(sid, []) == 0
    B_pad, T_pad, MB = 8, 32, 16
    for step in range(12):
        ids = [s for s in range(1, 6) if rng.random() < 0.8]
        ns = [int(rng.integers(1, 5)) for _ in ids]
        outs = []
        for p in pools:
            a = dict(positions=np.full(T_pad, 7, np.int32), slots=np.full(T_pad, 7, np.int32),
                     cu=np.full(B_pad + 1, 7, np.int32), ctx=np.full(B_pad, 7, np.int32),
                     bt=np.full((B_pad, MB), 7, np.int32), lidx=np.full(16, 7, np.int64))
            assert p.step_meta(ids, ns, B_pad, T_pad, MB, a["positions"], a["slots"], a["cu"], a["ctx"],
                               a["bt"], a["lidx"]) == 0
            outs.append(a)
        for k in outs[0]:
            assert np.array_equal(outs[0][k], outs[1][k]), (step, k)
    # exhausted pool / unknown sequence
    assert pools[1].step_meta([99], [1], B_pad, T_pad, MB, *[np.zeros(T_pad, np.int32)] * 2,
                              np.zeros(B_pad + 1, np.int32), np.zeros(B_pad, np.int32),
                              np.zeros((B_pad, MB), np.int32)) == -1


def test_hip_runtime_is_torchs_copy():
    """Direct HIP calls (CU-masked / prioritised streams, device flags) go to
    the libamdhip64 torch mapped, never to a second copy loaded by soname."""
    import torch

    from loqa_hub_amd.utils.hip_runtime import hip_runtime, mapped_hip_path
    lib = hip_runtime()
    assert os.path.realpath(mapped_hip_path()).startswith(
        os.path.realpath(os.path.dirname(os.path.dirname(torch.__file__)))) or "rocm" in mapped_hip_path()
    assert lib.hipStreamCreateWithPriority is not None
    with open("/proc/self/maps") as f:
        copies = {ln.split()[-1] for ln in f if "libamdhip64.so" in ln}
    assert len(copies) == 1, copies


def test_bench_cpu_smoke_hub_mode_bypass():
    """--mode hub --bypass: every bench relay is alone in its group, so no
    utterance waits for the arbitration window (the window here is 5 s: a
    run that waited would time out of the smoke's budget)."""
    out = _run([sys.executable, "bench.py", "--cpu-smoke", "--mode", "hub", "--steps", "1",
                "--warmup", "0", "--batch-per-gpu", "2", "--window-ms", "5000", "--bypass",
                "--window-steps", "0"])
    svc = out["hub"]["audio_service"]
    assert out["queue_success_rate"] == 1.0 and svc["processed"] == 2
    assert svc.get("bypassed", 0) == svc.get("windows", 0) > 0
