"""Per-step token budget and admission limits of the continuous-batching
schedulers (17+ sequences in a forced-literal run, or 33+ STT
arrivals feeding their SOT prompt, used to exceed the fused GEMMs' row limit
and fail every in-flight request)."""
import json
import numpy as np
import pytest
import torch

from loqa_hub_amd.engine.batching import plan_step
from loqa_hub_amd.engine.grammar import multi_command_schema
from loqa_hub_amd.llm.commands import parse_multi_command_response


def test_plan_step_budget_and_fairness():
    # under budget: everyone gets their feed, capped at max_q
    assert plan_step([1, 3, 20], 64, 8) == [1, 3, 8]
    # over budget: one token each first, then top-ups in order
    t = plan_step([8] * 10, 16, 8)
    assert sum(t) == 16 and all(x >= 1 for x in t) and t[0] == 7
    # more sequences than budget: a window of `budget` sequences, rotating
    t0 = plan_step([1] * 10, 4, 8, start=0)
    t1 = plan_step([1] * 10, 4, 8, start=4)
    assert t0 == [1, 1, 1, 1, 0, 0, 0, 0, 0, 0] and t1 == [0, 0, 0, 0, 1, 1, 1, 1, 0, 0]
    assert plan_step([], 8, 8) == []
    rng = np.random.default_rng(0)
    for _ in range(200):
        lens = rng.integers(1, 30, rng.integers(1, 80)).tolist()
        b, q = int(rng.integers(1, 65)), int(rng.integers(1, 17))
        t = plan_step(lens, b, q, int(rng.integers(0, 100)))
        assert sum(t) <= b and all(0 <= x <= min(n, q) for x, n in zip(t, lens))
        assert sum(1 for x in t if x) == min(b, len(lens))


def _wrap_steps(eng, name="decode_step"):
    seen = {"max_live": 0, "max_tokens": 0}
    orig = getattr(eng, name)

    def step(live):
        before = eng.stats.get("decode_tokens", 0)
        seen["max_live"] = max(seen["max_live"], len(live))
        out = orig(live)
        seen["max_tokens"] = max(seen["max_tokens"], eng.stats.get("decode_tokens", 0) - before)
        return out
    setattr(eng, name, step)
    return seen


def test_llm_scheduler_64_seqs_long_forced_runs_cpu():
    """max_seqs=64 (production HUB_MAX_BATCH), 80 submitted requests with
    4-command schemas: admission holds the overflow, every step stays under
    the token budget, and every request completes with valid JSON."""
    from loqa_hub_amd.engine.llm_engine import GenRequest, LLMEngine
    from loqa_hub_amd.models.configs import llama_config
    eng = LLMEngine(llama_config("test-tiny"), torch.device("cpu"), seed=0, max_seqs=64,
                    max_seq_len=512, use_graphs=False)
    assert eng.max_decode_q == 16 and eng.step_tokens == 64
    seen = _wrap_steps(eng)
    prompt = eng.tok.encode("turn on the lights and play music", bos=True)
    n_cmds = [1 + i % 4 for i in range(80)]
    reqs = [GenRequest(list(prompt), multi_command_schema(n)) for n in n_cmds]
    try:
        fut_a = eng.submit_batch(reqs[:70])     # oversize vs max_seqs: chunked
        fut_b = eng.submit_batch(reqs[70:])
        fut_a.result(timeout=600)
        fut_b.result(timeout=600)
    finally:
        eng.stop()
    assert seen["max_live"] <= 64
    assert 0 < seen["max_tokens"] <= 64
    for n, r in zip(n_cmds, reqs):
        assert r.done and len(parse_multi_command_response(r.output, "x").commands) == n
    assert eng.kv.pool.free_blocks() == eng.kv.num_blocks


def test_llm_generate_small_budget_cpu():
    """A budget below the live count: sequences sit steps out in turn."""
    from loqa_hub_amd.engine.llm_engine import GenRequest, LLMEngine
    from loqa_hub_amd.models.configs import llama_config
    eng = LLMEngine(llama_config("test-tiny"), torch.device("cpu"), seed=0, max_seqs=8,
                    max_seq_len=512, use_graphs=False)
    eng.step_tokens = 5
    seen = _wrap_steps(eng)
    reqs = [GenRequest(eng.tok.encode("dim the lights", bos=True), multi_command_schema(n))
            for n in (1, 2, 3, 4, 2, 3, 1, 4)]
    eng.generate(reqs)
    assert seen["max_tokens"] <= 5
    for n, r in zip((1, 2, 3, 4, 2, 3, 1, 4), reqs):
        assert len(parse_multi_command_response(r.output, "x").commands) == n


def test_stt_many_arrivals_under_budget_cpu():
    """More arrivals than the budget allows SOT prompts for: some sit a step
    out or feed part of the prompt; transcripts are unchanged."""
    from loqa_hub_amd.engine.stt_engine import STTEngine, STTRequest
    from loqa_hub_amd.engine.synthetic import make_batch
    from loqa_hub_amd.models.configs import whisper_config
    eng = STTEngine(whisper_config("test-whisper"), torch.device("cpu"), seed=0, max_batch=16)
    eng.step_tokens = 10
    seen = {"max_tokens": 0}
    orig = eng._step

    def step(live):
        seen["max_tokens"] = max(seen["max_tokens"], sum(len(r.feed) for r in live))
        return orig(live)
    eng._step = step
    utts = make_batch(0, 12, [1, 2, 3])
    reqs = [STTRequest(u.pcm, transcript=u.text) for u in utts]
    try:
        eng.submit_batch(reqs).result(timeout=600)
    finally:
        eng.stop()
    assert seen["max_tokens"] <= 10
    for r, u in zip(reqs, utts):
        assert r.text == u.text


def test_llm_inline_prefill_cpu(monkeypatch):
    """Inline prefill (prompt tail fed through the decode steps) gives the same
    greedy outputs as the separate prefill pass."""
    from loqa_hub_amd.engine.llm_engine import GenRequest, LLMEngine
    from loqa_hub_amd.models.configs import llama_config
    outs = {}
    for inline in ("0", "4096"):
        monkeypatch.setenv("LOQA_INLINE_PREFILL", inline)
        eng = LLMEngine(llama_config("test-tiny"), torch.device("cpu"), seed=0, max_seqs=8,
                        max_seq_len=512, use_graphs=False)
        assert eng.inline_prefill == int(inline)
        texts = ["turn on the lights and play music", "dim the kitchen lights", "hello there"]
        reqs = [GenRequest(eng.tok.encode(t, bos=True), multi_command_schema(n))
                for t, n in zip(texts, (2, 1, 1))]
        try:
            eng.submit_batch(reqs).result(timeout=300)
        finally:
            eng.stop()
        outs[inline] = [r.output for r in reqs]
        assert eng.stats["prefill_tokens"] > 0
    assert outs["0"] == outs["4096"]


def _run_sched(pipelined: bool, mispredict: float = 0.0):
    from loqa_hub_amd.engine.llm_engine import GenRequest, LLMEngine
    from loqa_hub_amd.models.configs import llama_config
    eng = LLMEngine(llama_config("test-tiny"), torch.device("cpu"), seed=0, max_seqs=6,
                    max_seq_len=512, use_graphs=False)
    eng.pipelined = pipelined
    texts = ["turn on the lights and play music", "dim the kitchen lights", "hello there",
             "turn off the tv then lock the door", "what time is it", "play music"]
    reqs = [GenRequest(eng.tok.encode(t, bos=True), multi_command_schema(n))
            for t, n in zip(texts, (2, 1, 1, 3, 1, 4))]
    try:
        eng.start()
        if pipelined:
            import time as _t
            while eng._pl is None:
                _t.sleep(0.01)
            eng._pl.force_mispredict = mispredict
        eng.submit_batch(reqs[:3]).result(timeout=300)
        eng.submit_batch(reqs[3:]).result(timeout=300)
    finally:
        eng.stop()
    assert eng.kv.pool.free_blocks() == eng.kv.num_blocks
    return [r.output for r in reqs], eng


def test_llm_pipelined_decode_matches_cpu():
    """Two steps in flight with device-fed tokens and predicted jump-forward
    literals: same greedy outputs as the synchronous loop, also when
    predictions are forced to fail (discard + KV rollback + re-feed)."""
    ref, _ = _run_sched(False)
    got, eng = _run_sched(True)
    assert got == ref
    assert eng._pl.stats["pl_spec"] > 0 and eng._pl.stats["pl_steps"] > 0
    got2, eng2 = _run_sched(True, mispredict=0.35)
    assert got2 == ref
    assert eng2._pl.stats["pl_discard"] > 0
    assert sorted(eng2._free_seq_slots) == list(range(6))


def _run_chunked(chunk: str, pipelined: bool, monkeypatch):
    from loqa_hub_amd.engine.llm_engine import GenRequest, LLMEngine
    from loqa_hub_amd.models.configs import llama_config
    monkeypatch.setenv("LOQA_CHUNK_PREFILL", chunk)
    monkeypatch.setenv("LOQA_INLINE_PREFILL", "0")     # every arrival takes a prompt pass
    eng = LLMEngine(llama_config("test-tiny"), torch.device("cpu"), seed=0, max_seqs=6,
                    max_seq_len=512, use_graphs=False)
    eng.pipelined = pipelined
    texts = ["turn on the lights and play music", "dim the kitchen lights", "hello there",
             "turn off the tv then lock the door", "what time is it", "play music"]
    reqs = [GenRequest(eng.tok.encode(t, bos=True), multi_command_schema(n))
            for t, n in zip(texts, (2, 1, 1, 3, 1, 4))]
    import time as _t
    try:
        eng.start()
        fa = eng.submit_batch(reqs[:3])
        t0 = _t.time()
        while not all(r.t_first for r in reqs[:3]) and _t.time() - t0 < 120:
            _t.sleep(0.002)           # the first batch is decoding: the second is chunked in
        fb = eng.submit_batch(reqs[3:])
        fa.result(timeout=300)
        fb.result(timeout=300)
    finally:
        eng.stop()
    assert eng.kv.pool.free_blocks() == eng.kv.num_blocks
    return [r.output for r in reqs], eng


@pytest.mark.parametrize("pipelined", [False, True])
def test_llm_chunked_prefill_matches_cpu(pipelined, monkeypatch):
    """Prompts arriving while others decode go in 5-token chunks, each chunk in
    one pass with the live sequences' next feeds (mixed steps): the same
    greedy outputs (and command counts) as whole prompt passes, the KV pool
    fully returned."""
    ref, _ = _run_chunked("0", pipelined, monkeypatch)
    got, eng = _run_chunked("5", pipelined, monkeypatch)
    assert eng.stats.get("mixed_steps", 0) >= 3
    # the live decoders' rows took the grouped decode attention (meta.split)
    assert eng.stats.get("mixed_split", 0) >= 1
    for a, b, n in zip(got, ref, (2, 1, 1, 3, 1, 4)):
        assert len(json.loads(a)["commands"]) == n
    assert got == ref


def test_synthetic_unique_utterances_outlast_the_base_pool():
    """A long bench run (hundreds of steps) draws more distinct one-command
    transcripts than the base pool holds (~320): the wider pool takes over
    instead of failing, every transcript stays distinct, and the early draws
    are those of the base generator (make_utterance), audio included."""
    import numpy as np

    from loqa_hub_amd.engine.synthetic import make_unique, make_utterance
    us = make_unique(3, [1] * 420)
    texts = [u.text for u in us]
    assert len(set(texts)) == 420
    first = make_utterance(3, 0, 1)
    assert us[0].text == first.text and np.array_equal(us[0].pcm, first.pcm)
    assert all(u.n_commands == 1 and len(u.pcm) > len(u.wake_pcm) for u in us)
