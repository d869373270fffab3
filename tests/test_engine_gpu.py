"""End-to-end engine checks on the GPU: the HIP path runs, graphs replay the
same tokens as eager execution, outputs parse with the expected command count."""
import json

import numpy as np
import pytest
import torch

from loqa_hub_amd.engine.grammar import multi_command_schema
from loqa_hub_amd.engine.llm_engine import GenRequest, LLMEngine
from loqa_hub_amd.engine.stt_engine import STTEngine, STTRequest
from loqa_hub_amd.models.configs import llama_config, whisper_config
from loqa_hub_amd.ops import _lib

pytestmark = pytest.mark.gpu


def test_native_loaded():
    assert _lib.available()


def _gen(eng, n_list):
    tok = eng.tok
    reqs = [GenRequest(tok.encode(f"Voice command: turn on the lights {i}", bos=True),
                       multi_command_schema(n, min_response_tokens=3)) for i, n in enumerate(n_list)]
    return eng.generate(reqs)


def test_llm_graphs_match_eager():
    cfg = llama_config("test-tiny")
    a = LLMEngine(cfg, "cuda", max_seqs=8, use_graphs=True)
    b = LLMEngine(cfg, "cuda", max_seqs=8, use_graphs=False)
    ra, rb = _gen(a, [1, 2, 3]), _gen(b, [1, 2, 3])
    for x, y, n in zip(ra, rb, [1, 2, 3]):
        assert x.output == y.output
        assert len(json.loads(x.output)["commands"]) == n


def _sched_outputs(eng, n_list, mispredict=0.0):
    tok = eng.tok
    reqs = [GenRequest(tok.encode(f"Voice command: turn on the lights {i}", bos=True),
                       multi_command_schema(n, min_response_tokens=3)) for i, n in enumerate(n_list)]
    eng.warmup_graphs()
    eng.start()
    try:
        if eng.pipelined:
            import time as _t
            while eng._pl is None:
                _t.sleep(0.01)
            eng._pl.force_mispredict = mispredict
        eng.submit_batch(reqs[:3]).result(timeout=120)
        eng.submit_batch(reqs[3:]).result(timeout=120)
    finally:
        eng.stop()
    return [r.output for r in reqs]


def test_llm_pipelined_decode_gpu():
    """Two graph-replayed steps in flight (device-fed tokens, zero-copy step
    I/O rings): same tokens as the synchronous graph loop, with and without
    forced prediction failures (discard + KV rollback)."""
    cfg = llama_config("test-tiny")
    n_list = [1, 2, 3, 4, 2, 1]
    a = LLMEngine(cfg, "cuda", max_seqs=8, use_graphs=True)
    a.pipelined = False
    ref = _sched_outputs(a, n_list)
    b = LLMEngine(cfg, "cuda", max_seqs=8, use_graphs=True)
    assert b.pipelined
    assert _sched_outputs(b, n_list) == ref
    assert b.stats["pl_spec"] > 0
    c = LLMEngine(cfg, "cuda", max_seqs=8, use_graphs=True)
    assert _sched_outputs(c, n_list, mispredict=0.3) == ref
    assert c.stats["pl_discard"] > 0
    for o, n in zip(ref, n_list):
        assert len(json.loads(o)["commands"]) == n


def test_llm_gpu_matches_cpu_reference_first_tokens():
    cfg = llama_config("test-tiny")
    g = LLMEngine(cfg, "cuda", max_seqs=4, use_graphs=False)
    c = LLMEngine(cfg, "cpu", max_seqs=4)
    # same weights on both
    c.weights.__dict__.update({k: (v.cpu() if torch.is_tensor(v) else v)
                               for k, v in g.weights.__dict__.items()})
    c.weights.layers = [{k: t.cpu() for k, t in L.items()} for L in g.weights.layers]
    c.weights.decode_layers = [{k: t.cpu() for k, t in L.items()} for L in g.weights.decode_layers]
    c.weights.cos_sin = g.weights.cos_sin.cpu()
    c.model.w = c.weights
    rg, rc = _gen(g, [2]), _gen(c, [2])
    # bf16 kernels vs fp32 reference may diverge late; the first sampled decisions agree
    assert rg[0].grammar.emitted[:8] == rc[0].grammar.emitted[:8]


def test_stt_whisper_tiny_gpu():
    e = STTEngine(whisper_config("whisper-tiny"), "cuda", max_batch=4)
    reqs = [STTRequest((np.random.randn(32000) * 2000).astype(np.int16), transcript="turn on the lights"),
            STTRequest((np.random.randn(8000) * 2000).astype(np.int16), transcript="hello there")]
    e.transcribe(reqs)
    assert reqs[0].text == "turn on the lights"
    assert reqs[1].text == "hello there"
    assert reqs[0].rms > 0


def _whisper_first_logits(eng, pcms):
    from loqa_hub_amd.models.whisper import decode_step_fast
    reqs = [STTRequest(p) for p in pcms]
    audio, _ = eng.upload(reqs)
    eng.cross_kv(eng.model.encode(audio))
    for i, r in enumerate(reqs):
        r.seq_id = eng._next
        r.slot = i
        r.feed = list(eng.sot)
        eng._next += 1
        eng.kv.pool.add_seq(r.seq_id, [])
    max_q, host = eng._host_meta(reqs, 2, 16)
    dev = eng._dev(host)
    if eng.fast_decode:
        lg = decode_step_fast(eng.model, dev["tokens"], dev["positions"], dev["slots"],
                              dev["cu_q"], dev["ctx_lens"], dev["block_tables"], max_q, eng.kv.k,
                              eng.kv.v, eng.xkv, dev["enc_starts"], dev["enc_lens"],
                              dev["logit_idx"], eng.ws, eng.self_splits)
        return lg[:2, : eng.cfg.vocab_size].float()
    T = int(host["cu_q"][2])
    return eng.model.decode_step(
        dev["tokens"][:T], dev["positions"][:T], dev["slots"][:T], dev["cu_q"][:3],
        dev["ctx_lens"][:2], dev["block_tables"][:2], max_q, int(host["ctx_lens"].max()),
        eng.kv.k, eng.kv.v, eng.xkv, dev["enc_starts"][:2], dev["enc_lens"][:2],
        dev["logit_idx"][:2], eng.ws).float()


@pytest.mark.parametrize("name", ["whisper-tiny", "whisper-base"])
def test_whisper_fast_decode_matches_eager_gpu(name):
    cfg = whisper_config(name)
    rng = np.random.default_rng(0)
    pcms = [(rng.standard_normal(24000) * 3000).astype(np.int16),
            (rng.standard_normal(40000) * 3000).astype(np.int16)]
    fast = STTEngine(cfg, "cuda", seed=1, max_batch=4, fast_decode=True)
    eager = STTEngine(cfg, "cuda", seed=1, max_batch=4, fast_decode=False)
    a, b = _whisper_first_logits(fast, pcms), _whisper_first_logits(eager, pcms)
    err = (a - b).abs().max().item()
    assert err <= 2e-2 * b.abs().max().item() + 1e-3, err


def test_whisper_graphs_match_eager_fast():
    cfg = whisper_config("whisper-tiny")
    rng = np.random.default_rng(1)
    pcms = [(rng.standard_normal(n) * 3000).astype(np.int16) for n in (16000, 48000, 30000)]
    outs = []
    for graphs in (True, False):
        e = STTEngine(cfg, "cuda", seed=2, max_batch=4, use_graphs=graphs)
        reqs = [STTRequest(p, max_new_tokens=12) for p in pcms]
        e.transcribe(reqs)
        outs.append([r.tokens for r in reqs])
    assert outs[0] == outs[1]


def test_vits_tts_gpu():
    from loqa_hub_amd.engine.tts_engine import VitsTTSEngine
    from loqa_hub_amd.models.configs import VITS_CONFIGS
    e = VitsTTSEngine(VITS_CONFIGS["vits-ljs"], "cuda")
    outs = e.synthesize_batch(["Turning on the kitchen lights.", "Done."])
    assert len(outs) == 2 and outs[0].dtype == np.int16
    assert outs[0].size % 256 == 0 and outs[0].size > outs[1].size > 0
    assert np.abs(outs[0].astype(np.float32)).mean() > 100


def test_vits_graph_runner_matches_eager_gpu():
    """Bucketed two-graph VITS replay (text graph per (batch, symbols), audio
    graph per (batch, symbols, frames); seed and length scale as device
    scalars) gives the eager synthesis at the same frame count bitwise, replay
    after replay with fresh seeds."""
    from loqa_hub_amd.models.configs import VITS_CONFIGS
    from loqa_hub_amd.models.vits import VitsGraphRunner, VitsModel, VitsWeights, text_to_ids
    cfg = VITS_CONFIGS["test-vits"]
    m = VitsModel(VitsWeights(cfg, "cuda", seed=5))
    texts = ["Turning on the kitchen lights.", "Done.", "Playing jazz in the bedroom now."]
    ids_l = [text_to_ids(t, cfg.n_symbols) for t in texts]
    T = max(len(i) for i in ids_l)
    ids = torch.zeros(len(ids_l), T, dtype=torch.int64, device="cuda")
    for b, i in enumerate(ids_l):
        ids[b, :len(i)] = torch.tensor(i, device="cuda")
    lens = torch.tensor([len(i) for i in ids_l], dtype=torch.int32, device="cuda")
    st = torch.cuda.Stream()
    with torch.cuda.stream(st), torch.inference_mode():
        run = VitsGraphRunner(m, "cuda")
        run.MAX_AUDIO_GRAPHS = 1          # every new frame bucket evicts the last one
        outs = []
        for seed, ls in ((3, 1.0), (9, 1.0), (9, 2.0), (5, 1.0)):
            pg, ng = run.synthesize(ids, lens, seed=seed, length_scale=ls)
            pg, ng = pg.clone(), ng.clone()
            pe, ne = m.synthesize(ids, lens, seed=seed, length_scale=ls, frame_step=run.F_STEP)
            st.synchronize()
            assert torch.equal(ng, ne) and pg.shape == pe.shape
            assert torch.equal(pg, pe), (pg.float() - pe.float()).abs().max().item()
            outs.append(pg)
        one, n1 = run.synthesize(ids[1:2], lens[1:2], seed=3)
        st.synchronize()
    assert run.stats["replays"] == 5 and run.stats["eager"] == 0
    assert run.stats["evicted"] >= 1           # replays after an eviction still match eager
    assert not torch.equal(outs[0], outs[1])          # a new seed draws new noise
    assert int(n1[0]) == int(ne[1])            # a row alone: same frame count
    assert np.abs(one.float().cpu().numpy()).mean() > 50


def test_stt_continuous_batching_gpu():
    """Graph-replayed Whisper decode with requests joining a running batch
    (per-request cross-attention slots) equals the one-shot batch."""
    import time as _t
    cfg = whisper_config("whisper-tiny")
    rng = np.random.default_rng(1)
    pcms = [(rng.standard_normal(16000 * (i + 1)) * 3000).astype(np.int16) for i in range(3)]
    ref = STTEngine(cfg, "cuda", seed=1, max_batch=4)
    solo = [STTRequest(p, max_new_tokens=8) for p in pcms]
    ref.transcribe(solo)
    eng = STTEngine(cfg, "cuda", seed=1, max_batch=4)
    a = [STTRequest(p, max_new_tokens=8) for p in pcms[:2]]
    b = [STTRequest(pcms[2], max_new_tokens=8)]
    fa = eng.submit_batch(a)
    _t.sleep(0.02)
    fb = eng.submit_batch(b)
    fa.result(timeout=120)
    fb.result(timeout=120)
    eng.stop()
    for got, want in zip(a + b, solo):
        assert got.tokens == want.tokens


@pytest.mark.parametrize("streaming", [True, False])
def test_hub_server_gpu_served(tmp_path, streaming):
    """The composed hub with the ON-DEVICE processor: a relay streams audio over
    real gRPC, the arbitration winner goes through the GPU pipeline (Whisper-
    tiny encoder + decoder graphs, constrained Llama decode, command queue on
    NATS), the bridge runs on that decode, the reply is spoken by on-GPU VITS -
    progressively, phrase by phrase, when streaming is enabled - and published
    on NATS audio.<relay>; the voice event lands in SQLite and /api; the
    streaming routes answer from the composed streaming subsystem. (With this
    test's small models the whole decode is shorter than one VITS synthesis,
    so audio-before-decode-end is measured on config 5:
    scripts/bench_configs.py first_audio_before_decode_done.)"""
    from tests.test_hub_served import _check_served, _served
    res = _served(tmp_path, "cuda:0", streaming=streaming, llm="test-tiny", stt="whisper-tiny",
                  tts_model="test-vits")
    _check_served(*res, streaming=streaming, relays=("kitchen-relay",))


def test_hub_server_gpu_served_dp_shared(tmp_path):
    """The served DP hub on the GPU: two worker processes (sharing cuda:0
    here; one per GPU on a node), each with the full composition - its own
    NATS connection, VITS, bridge, progressive speech, pinned PCM staging of
    the raw PCM16 the front end ships."""
    from tests.test_hub_served import _check_served, _served
    relays = ("kitchen-relay", "bedroom-relay")
    res = _served(tmp_path, "cuda:0", streaming=True, llm="test-tiny", stt="whisper-tiny",
                  tts_model="test-vits", dp=2, relays=relays)
    _check_served(*res, streaming=True, relays=relays)
    assert sorted(res[4]["dp_workers"]) == [0, 1]


@pytest.mark.parametrize("model", ["tinyllama", "llama3-8b"])
def test_llm_prefill_hw_matches_hipblaslt_gpu(monkeypatch, model):
    """Prefill on the hand-written GEMMs (ops.proj: qkv, o + residual,
    gate|up + SwiGLU, down + residual; in-launch K reduction) vs plain
    hipBLASLt GEMMs + rmsnorm: final hidden rows of a 300-token prompt and the
    KV rows agree."""
    from loqa_hub_amd.models import llama as llama_mod
    cfg = llama_config(model, n_layers=4) if model == "llama3-8b" else llama_config(model)
    eng = LLMEngine(cfg, "cuda", max_seqs=2, max_seq_len=512, use_graphs=False)
    g = torch.Generator().manual_seed(4)
    toks = torch.randint(3, 30000, (300,), generator=g).tolist()
    r = GenRequest(toks, multi_command_schema(1))
    eng.submit(r)
    max_q, max_ctx, host = eng._meta([r], [r.feed], decode=False)
    dev = eng._to_device(host)
    meta = eng._build_meta(dev, max_q, max_ctx, False)
    outs, kvs = {}, {}
    for key, on in (("hw", True), ("blas", False)):
        monkeypatch.setattr(llama_mod, "PREFILL_HW", on)
        outs[key] = eng.model.forward(meta, eng.kv.k, eng.kv.v, eng.attn_ws).float()
        kvs[key] = (eng.kv.k[-1].float().clone(), eng.kv.v[-1].float().clone())
    for key in ("hw",):
        rel = float((outs[key] - outs["blas"]).norm() / outs["blas"].norm())
        assert torch.isfinite(outs[key]).all() and rel < 4e-2, (key, rel)
        for a, b in zip(kvs[key], kvs["blas"]):
            assert float((a - b).norm() / b.norm()) < 4e-2, key


def test_prefill_logits_on_skinny_lm_head_gpu():
    """The prompt pass's sampling rows go through the decode steps'
    weight-streaming lm_head (no hipBLASLt): f32 logits agree with the bf16
    hipBLASLt GEMM and give the same argmax."""
    cfg = llama_config("tinyllama")
    eng = LLMEngine(cfg, "cuda", max_seqs=2, max_seq_len=256, use_graphs=False)
    w = eng.weights
    for B in (1, 3, 16, 20):
        h = torch.randn(B, cfg.d_model, device="cuda").bfloat16()
        got = eng.model.logits(h).float()
        ref = torch.nn.functional.linear(h, w.lm_head).float()
        assert got.shape == ref.shape == (B, w.v)
        rel = float((got - ref).norm() / ref.norm())
        assert rel < 1e-2, (B, rel)
        top2 = ref.topk(2, dim=-1).values
        tie = (top2[:, 0] - top2[:, 1]) < 0.05 * ref.abs().max()
        assert bool(((got.argmax(-1) == ref.argmax(-1)) | tie).all())


def _to_cpu(obj, seen=None):
    """Deep copy of a weights object with every tensor on the CPU."""
    import copy
    if torch.is_tensor(obj):
        return obj.detach().cpu()
    if isinstance(obj, dict):
        return {k: _to_cpu(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to_cpu(v) for v in obj)
    if hasattr(obj, "__dict__") and not isinstance(obj, type) and \
            not getattr(type(obj), "__dataclass_params__", None):
        c = copy.copy(obj)
        c.__dict__ = {k: _to_cpu(v) for k, v in obj.__dict__.items()}
        return c
    return obj       # configs (frozen dataclasses), scalars


def test_vits_gpu_matches_fp32_reference():
    """Full VITS on the HIP kernels vs the fp32 PyTorch reference (ops/reference.py
    path on the CPU) with the SAME weights, stage by stage: text encoder
    statistics, durations, the reverse flow and the HiFi-GAN waveform."""
    from loqa_hub_amd.models.configs import VITS_CONFIGS
    from loqa_hub_amd.models.vits import VitsModel, VitsWeights, text_to_ids
    cfg = VITS_CONFIGS["test-vits"]
    gw = VitsWeights(cfg, "cuda", seed=3)
    gm, cm = VitsModel(gw), VitsModel(_to_cpu(gw))
    texts = ["Turning on the kitchen lights.", "Playing some jazz now."]
    ids = [text_to_ids(t, cfg.n_symbols) for t in texts]
    T = max(len(i) for i in ids)
    arr = torch.zeros(len(ids), T, dtype=torch.int64)
    for b, i in enumerate(ids):
        arr[b, :len(i)] = torch.tensor(i)
    lens = torch.tensor([len(i) for i in ids], dtype=torch.int32)

    def rel(a, b):
        a, b = a.float().cpu(), b.float().cpu()
        return float((a - b).norm() / b.norm().clamp_min(1e-6))
    with torch.inference_mode():
        sg, xg = gm.encode_text(arr.cuda(), lens.cuda())
        sc, xc = cm.encode_text(arr, lens)
        assert rel(sg, sc) < 3e-2 and rel(xg, xc) < 3e-2, (rel(sg, sc), rel(xg, xc))
        dg, dc = gm.durations(xg, lens.cuda(), 1.0).cpu(), cm.durations(xc, lens, 1.0)
        assert (dg == dc).float().mean() >= 0.9
        # the same latent through the reverse flow and the vocoder on both paths
        cum = torch.cumsum(dc, dim=1, dtype=torch.int32)
        flen = cum[:, -1].contiguous()
        F = int(flen.max())
        z = torch.randn(len(ids), F, cfg.inter_channels, generator=torch.Generator().manual_seed(0))
        z = (z * 0.5).to(torch.bfloat16)
        zg, zc = gm.flow_reverse(z.cuda(), flen.cuda()), cm.flow_reverse(z, flen)
        assert rel(zg, zc) < 5e-2, rel(zg, zc)
        hop = 1
        for r in cfg.upsample_rates:
            hop *= r
        pg = gm.decode(zc.cuda(), (flen * hop).to(torch.int32).cuda()).float().cpu()
        pc = cm.decode(zc, (flen * hop).to(torch.int32)).float()
        assert pg.shape == pc.shape
        assert rel(pg, pc) < 0.1, rel(pg, pc)
        assert pc.abs().mean() > 50


def test_pinned_pcm_stager_upload_gpu():
    """Relay chunks appended into a pinned stager slot (odd trailing bytes
    dropped per chunk, as the reference) reach HBM byte-identical through the
    H2D stream, and the padded convert kernel yields x / 32767 with zeros past
    the utterance; a numpy request in the same batch is staged on the fly."""
    from loqa_hub_amd.engine.stt_engine import N_SAMPLES, STTRequest
    eng = STTEngine(whisper_config("whisper-tiny"), "cuda", max_batch=4)
    rng = np.random.default_rng(7)
    chunks = [rng.integers(0, 256, size=n, dtype=np.uint8).tobytes() for n in (3201, 640, 17, 9600)]
    slot = eng.new_pcm_slot()
    for c in chunks:
        slot.append(c)
    expect = np.frombuffer(b"".join(c[: len(c) & ~1] for c in chunks), "<i2")
    other = (rng.standard_normal(5000) * 3000).astype(np.int16)
    reqs = [STTRequest(np.zeros(0, np.int16), staged=slot), STTRequest(other)]
    audio, sumsq = eng.upload(reqs)
    torch.cuda.synchronize()
    a = audio.cpu().numpy()
    assert a.shape == (2, N_SAMPLES)
    assert np.array_equal(np.round(a[0, :expect.size] * 32767.0).astype(np.int64), expect.astype(np.int64))
    assert not a[0, expect.size:].any() and not a[1, other.size:].any()
    assert np.array_equal(np.round(a[1, :other.size] * 32767.0).astype(np.int64), other.astype(np.int64))
    ref = (expect.astype(np.float64) / 32767.0) ** 2
    assert abs(float(sumsq[0]) - ref.sum()) <= 1e-3 * ref.sum()
    assert reqs[0].staged is None and slot.released


def test_gpu_streaming_backend_joins_continuous_batch():
    """The streaming parser's GPU backend submits into the running continuous
    batch (submit_batch) - two concurrent sessions share decode steps."""
    import asyncio

    from loqa_hub_amd.streaming.parser import GPUStreamingBackend, StreamingCommandParser
    eng = LLMEngine(llama_config("test-tiny"), "cuda", max_seqs=4, max_seq_len=512)
    eng.warmup_graphs()

    async def go():
        p = StreamingCommandParser(GPUStreamingBackend(eng), None)
        rs = await asyncio.gather(*[p.parse_command_streaming(t) for t in
                                    ("turn on the kitchen lights", "play some jazz")])
        out = []
        for r in rs:
            toks = [t async for t in r.token_stream]
            out.append((toks, await asyncio.wait_for(r.final_command.get(), 60)))
        return out
    try:
        out = asyncio.run(go())
    finally:
        eng.stop()
    assert all(len(t) > 3 and c.intent for t, c in out)
    assert eng.stats["decode_steps"] > 0


def test_bench_dp2_shared_gpu():
    """Two bench ranks on the one GPU of a test box (LOQA_DIST_SHARE_GPU=1:
    gloo control plane, every rank on cuda:0): per-rank GPU pipelines with
    graphs, the node's one NATS broker, records gathered to rank 0. The RCCL
    collectives of a real multi-GPU run are the only part not exercised."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", LOQA_DIST_SHARE_GPU="1", LOQA_NO_TUNE="1",
               OMP_NUM_THREADS="2")
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "2", "--master-addr", "127.0.0.1", "--master-port",
                        "29571", "bench.py", "--stt", "test-whisper", "--llm", "test-tiny",
                        "--gpus", "2", "--steps", "1", "--warmup", "1", "--batch-per-gpu", "2"],
                       cwd=root, env=env, capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2"
    assert out["config"]["global_batch"] == 4 and out["queue_success_rate"] == 1.0
    assert out["command_count_match_rate"] == 1.0


def test_llm_chunked_prefill_gpu(monkeypatch):
    """Prompts arriving while others decode go in chunks, each chunk in one
    pass with the live sequences' next feeds (hand-written prompt-pass GEMMs),
    after a drain of the pipelined graph steps: every request completes with
    the expected command count, KV blocks and sequence slots all returned."""
    import time as _t
    monkeypatch.setenv("LOQA_CHUNK_PREFILL", "16")
    monkeypatch.setenv("LOQA_INLINE_PREFILL", "0")
    cfg = llama_config("test-tiny")
    eng = LLMEngine(cfg, "cuda", max_seqs=8, use_graphs=True)
    assert eng.chunk_prefill == 16 and eng.pipelined
    n_list = [2, 3, 1, 4, 2, 1]
    tok = eng.tok
    reqs = [GenRequest(tok.encode(f"Voice command: turn on the lights {i}", bos=True),
                       multi_command_schema(n, min_response_tokens=3)) for i, n in enumerate(n_list)]
    eng.warmup_graphs()
    eng.start()
    try:
        fa = eng.submit_batch(reqs[:3])
        t0 = _t.time()
        while not all(r.t_first for r in reqs[:3]) and _t.time() - t0 < 60:
            _t.sleep(0.001)
        fb = eng.submit_batch(reqs[3:])
        fa.result(timeout=120)
        fb.result(timeout=120)
    finally:
        eng.stop()
    assert eng.stats.get("mixed_steps", 0) > 0
    for r, n in zip(reqs, n_list):
        assert len(json.loads(r.output)["commands"]) == n
    assert eng.kv.pool.free_blocks() == eng.kv.num_blocks
    assert sorted(eng._free_seq_slots) == list(range(8))


def test_placed_stream_slot_gpu():
    """Every serving stream is the pool stream at its fixed slot, whatever
    drew pool streams before it, and runs work."""
    from loqa_hub_amd.utils.streams import DEFAULT_SLOTS, init_pools, placed_stream, pool_slot
    dev = torch.device("cuda", 0)
    init_pools(dev)
    for _ in range(5):
        torch.cuda.Stream(dev)            # move the pool cursor
    s = placed_stream(dev, "llm")
    assert pool_slot(s, dev, 0) == DEFAULT_SLOTS["llm"]
    h = placed_stream(dev, "stt", -1)
    assert pool_slot(h, dev, -1) == DEFAULT_SLOTS["stt"]
    with torch.cuda.stream(s):
        x = torch.full((4096,), 2.0, device=dev)
        y = (x * x).sum()
    s.synchronize()
    assert y.item() == 4.0 * 4096


def test_stt_suppression_checkpoint_tokenizer_gpu(tmp_path):
    """The suppression mask of a checkpoint tokenizer on the graph-replayed
    Whisper decode (masked argmax kernel, one mask row for every sequence)."""
    from test_tokenizer_hf import WHISPER_SPECIALS, _byte_level
    from loqa_hub_amd.engine.synthetic import make_batch
    from loqa_hub_amd.engine.tokenizer import load_tokenizer
    f = _byte_level(str(tmp_path / "whisper"), vocab=3000, specials=WHISPER_SPECIALS)
    with open(tmp_path / "whisper" / "generation_config.json", "w") as fh:
        json.dump({"suppress_tokens": list(range(300, 2900))}, fh)
    tok = load_tokenizer(f, 4096)
    eng = STTEngine(whisper_config("test-whisper"), "cuda", seed=0, max_batch=4, tokenizer=tok)
    utts = make_batch(0, 3, [1, 2])
    reqs = [STTRequest(u.pcm, max_new_tokens=12) for u in utts]
    eng.transcribe(reqs)
    allowed = set(tok.sampling_mask(keep=(eng.eot,)).nonzero().flatten().tolist())
    toks = [t for r in reqs for t in r.tokens]
    assert toks and set(toks) <= allowed


def _rel_max(a: torch.Tensor, b: torch.Tensor) -> float:
    return float((a - b).abs().max() / b.abs().max())


def test_llama3_8b_fused_graph_decode_vs_fp32_gpu():
    """Llama-3-8B shapes (4 layers + the full 128k lm_head)
    through the fused, graph-replayed decode step, teacher-forced for 32
    steps after a 24-token prompt (fed 8 tokens per fused step), against an
    fp32 torch forward on the same weights (ops.reference.llama_forward_ref):
    every step's logits within 2e-2 of the fp32 logits' max (relative), and
    the greedy choice equal except at near-ties."""
    from loqa_hub_amd.ops import reference as ref
    cfg = llama_config("llama3-8b", n_layers=4)
    eng = LLMEngine(cfg, "cuda", seed=3, max_seqs=2, max_seq_len=256, use_graphs=True)
    w, P, STEPS = eng.weights, 24, 32
    g = torch.Generator().manual_seed(7)
    toks = torch.randint(3, cfg.vocab_size, (P + STEPS,), generator=g).tolist()
    r = GenRequest(toks[:P], [])
    r.seq_id = 1
    eng.kv.pool.add_seq(1, [])

    def fused(feed, dev=None):
        max_q, _, host = eng._meta([r], [feed], True, 1, 16)
        if dev is None:
            dev = eng._to_device(host)
        else:
            for k, a in host.items():
                dev[k].copy_(torch.from_numpy(a))
        return dev, eng._build_meta(dev, max_q, 256, True)
    for c in range(0, P, 8):                     # the prompt, 8 rows per fused step
        _, meta = fused(toks[c:c + 8])
        eng.model.forward_decode_fused(meta, eng.kv.k, eng.kv.v, eng.attn_ws, eng.scratch)
    dev, meta = fused([toks[P]])                 # step 0 (runs once here as the warm-up)
    eng.model.forward_decode_fused(meta, eng.kv.k, eng.kv.v, eng.attn_ws, eng.scratch)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        out = eng.model.forward_decode_fused(meta, eng.kv.k, eng.kv.v, eng.attn_ws, eng.scratch)
    errs, agree = [], 0
    for s in range(STEPS):
        if s > 0:
            fused([toks[P + s]], dev)
        graph.replay()
        torch.cuda.synchronize()
        got = out[0].float()
        want = ref.llama_forward_ref(w, toks[: P + s + 1])[-1]
        errs.append(_rel_max(got, want))
        top2 = want.topk(2).values
        agree += int(got.argmax() == want.argmax() or float(top2[0] - top2[1]) < 2e-2 * float(
            want.abs().max()))
    print("llama3-8b x4 fused graph decode: max rel logit err per step", max(errs))
    assert max(errs) <= 2e-2, errs
    assert agree == STEPS


def test_whisper_large_v3_fused_graph_decode_vs_fp32_gpu():
    """Whisper-large-v3 decoder shapes (2 layers, d 1280, 20
    heads, 51866 vocab) through the fused, graph-replayed decode step with
    cross-attention over 1500 encoder rows, teacher-forced (the 4-token SOT
    prompt, then 16 one-token steps), against an fp32 torch decoder on the
    same weights (ops.reference.whisper_decoder_ref): per-step logits within
    2e-2 relative."""
    from loqa_hub_amd.models.whisper import decode_step_fused
    from loqa_hub_amd.ops import reference as ref
    cfg = whisper_config("whisper-large-v3", enc_layers=1, dec_layers=2)
    eng = STTEngine(cfg, "cuda", seed=2, max_batch=2, use_graphs=False)
    assert eng.fused
    g = torch.Generator().manual_seed(5)
    enc = torch.randn(cfg.n_audio_ctx, cfg.d_model, generator=g).to("cuda", torch.bfloat16)
    eng.cross_kv(enc)
    toks = list(eng.sot) + torch.randint(0, 50000, (16,), generator=g).tolist()
    r = STTRequest(np.zeros(160, np.int16))
    r.seq_id, r.slot = 1, 0
    eng.kv.pool.add_seq(1, [])

    def step(feed, dev=None):
        r.feed = feed
        max_q, host = eng._host_meta([r], 1, 16)
        if dev is None:
            dev = eng._dev(host)
        else:
            for k, a in host.items():
                dev[k].copy_(torch.from_numpy(a))
        return dev, max_q

    def fwd(dev, max_q):
        return decode_step_fused(eng.model, dev["tokens"], dev["positions"], dev["slots"],
                                 dev["cu_q"], dev["ctx_lens"], dev["block_tables"], max_q,
                                 eng.kv.k, eng.kv.v, eng.xkv, dev["enc_starts"], dev["enc_lens"],
                                 dev["logit_idx"], eng.ws, eng.scratch, eng.self_splits,
                                 eng.SPLIT_KEYS, eng.cross_split_keys)
    V, n0 = cfg.vocab_size, len(eng.sot)
    errs = []
    dev, mq = step(toks[:n0])                     # the SOT prompt, eager
    got = fwd(dev, mq)[0, :V].float()
    errs.append(_rel_max(got, ref.whisper_decoder_ref(eng.weights, toks[:n0], enc)[-1]))
    dev, mq = step([toks[n0]])                    # first one-token step (warm-up run)
    fwd(dev, mq)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        out = fwd(dev, mq)
    for s in range(n0, len(toks)):
        if s > n0:
            step([toks[s]], dev)
        graph.replay()
        torch.cuda.synchronize()
        want = ref.whisper_decoder_ref(eng.weights, toks[: s + 1], enc)[-1]
        errs.append(_rel_max(out[0, :V].float(), want))
    print("whisper-large-v3 x2 fused graph decode: max rel logit err per step", max(errs))
    assert max(errs) <= 2e-2, errs
