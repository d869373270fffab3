"""Tensor-parallel serving on the GPU (BASELINE config 5's layout).

The round-end box has one MI355X, so the TP ranks share cuda:0 (as in
test_custom_allreduce_gpu.py): every collective is the real custom IPC kernel
(row-parallel residual all-reduce, vocab-parallel argmax combine), the decode
steps are captured HIP graphs replayed in lock step, and the scheduler of every
follower replays the leader's arrivals from the shared-memory control ring. Only
the physical links differ from an 8-GPU node.

Checks, for TP=2, 4 and 8 of Llama-3-8B's shapes (4 layers, to keep the test
short) against TP=1 on the same seed (the counter-based init gives every TP
degree the same model):

* teacher-forced decode logits through the fused TP step (f32 partials, one
  reduce-scatter / all-gather residual kernel per projection): close to TP=1,
  and the greedy token identical at every step whose TP=1 top-2 margin is not
  a near tie (f32 split-K partial sums associate differently across TP
  degrees, so a bitwise-equal logit is not expected - a tie can flip);
* the lock-step serving loop: every rank runs the same decode steps with no
  collective error, and the constrained outputs are valid with the same
  command counts as TP=1."""
import json
import sys
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _reqs(eng, wave):
    from loqa_hub_amd.engine.grammar import multi_command_schema
    from loqa_hub_amd.engine.llm_engine import GenRequest
    out = []
    for i, n in enumerate((1, 3, 2)):
        text = f"wave {wave} utterance {i}: turn on the kitchen lights and play some jazz"
        out.append(GenRequest(eng.tok.encode(text, bos=True),
                              multi_command_schema(n, min_response_tokens=3)))
    return out


def _teacher_forced_logits(eng, steps: int = 24):
    """Prefill 3 fixed prompts, then ``steps`` decode steps feeding a fixed
    token per sequence through the fused decode step; full-vocab logits
    [steps + 1, 3, V] (the TP shards gathered over the CPU group)."""

    from loqa_hub_amd.engine.llm_engine import GenRequest
    prompts = [list(range(100 + 7 * i, 140 + 7 * i)) for i in range(3)]
    reqs = [GenRequest(p, []) for p in prompts]
    for r in reqs:
        r.seq_id = eng._next_id
        eng._next_id += 1
        eng.kv.pool.add_seq(r.seq_id, [])

    def gather(local):
        local = local.float().cpu()
        if eng.tp.world == 1:
            return local
        parts = [torch.empty_like(local) for _ in range(eng.tp.world)]
        dist.all_gather(parts, local, group=eng.tp.group)
        return torch.cat(parts, dim=1)

    out = []
    max_q, max_ctx, host = eng._meta(reqs, prompts, decode=False)
    meta = eng._build_meta(eng._to_device(host), max_q, max_ctx, False)
    out.append(gather(eng.model.logits(eng.model.forward(meta, eng.kv.k, eng.kv.v, eng.attn_ws))))
    for t in range(steps):
        feeds = [[(1000 + 37 * t + 11 * i) % 120000] for i in range(3)]
        max_q, max_ctx, host = eng._meta(reqs, feeds, True, 3, 16)
        meta = eng._build_meta(eng._to_device(host), max_q, max_ctx, True)
        lg = eng.model.forward_decode_fused(meta, eng.kv.k, eng.kv.v, eng.attn_ws, eng.scratch)
        out.append(gather(lg[:3]))
    for r in reqs:
        eng.kv.pool.free_seq(r.seq_id)
    torch.cuda.synchronize()
    return torch.stack(out)


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if world >= 8:
        # 8 processes x HIP's 4 hardware queues oversubscribe the GPU's queue
        # slots and the ranks get time-sliced (~28x slower steps,
        # profiles/r3_tp8_share_hwq.txt); read at HIP init (first GPU call)
        os.environ["GPU_MAX_HW_QUEUES"] = "1"
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        from loqa_hub_amd.engine.llm_engine import LLMEngine
        from loqa_hub_amd.models.configs import llama_config
        from loqa_hub_amd.models.llama import TPGroup
        from loqa_hub_amd.parallel.tp_control import TPControl
        cfg = llama_config("llama3-8b", n_layers=4)
        tp = TPGroup.create(rank, world, dist.group.WORLD, device=dev)
        eng = LLMEngine(cfg, dev, max_seqs=8, max_seq_len=512, tp=tp, seed=11)
        if world > 1:
            eng.tp_ctl = TPControl(rank, world, f"gputest{port}", dist.group.WORLD)
        logits = _teacher_forced_logits(eng)
        if rank == 0:
            torch.save(logits, os.path.join(out_dir, f"tp{world}_logits.pt"))
        n_graphs = eng.warmup_graphs()
        res = {"graphs": n_graphs}
        if rank == 0:
            outs = []
            for wave in range(2):
                futs = [eng.submit_batch([r]) for r in _reqs(eng, wave)]
                outs += [r.output for f in futs for r in f.result(timeout=300)]
            eng.stop()
            res["outs"] = outs
        else:
            eng.follow()
        torch.cuda.synchronize()
        res["decode_steps"] = eng.stats["decode_steps"]
        if tp.car is not None:
            res["car_error"] = tp.car.error()
            res["car_calls"] = tp.car.calls
            res["car_fallbacks"] = tp.car.fallbacks
        with open(os.path.join(out_dir, f"tp{world}_r{rank}.json"), "w") as f:
            json.dump(res, f)
        if eng.tp_ctl is not None:
            eng.tp_ctl.close()
    finally:
        dist.destroy_process_group()


def _run(world, out_dir):
    ctx = mp.get_context("spawn")
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, out_dir)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=600)
    alive = [p for p in procs if p.is_alive()]
    for p in alive:
        p.kill()
    assert not alive, f"TP={world} ranks hung"
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    return [json.load(open(os.path.join(out_dir, f"tp{world}_r{r}.json"))) for r in range(world)]


def test_tp_decode_matches_tp1(tmp_path):
    ref = _run(1, str(tmp_path))[0]
    assert ref["graphs"] > 0 and len(ref["outs"]) == 6
    ref_logits = torch.load(tmp_path / "tp1_logits.pt", weights_only=True)
    for world in (2, 4, 8):
        res = _run(world, str(tmp_path))
        lg = torch.load(tmp_path / f"tp{world}_logits.pt", weights_only=True)
        scale = ref_logits.abs().max().item()
        err = (lg - ref_logits).abs().max().item()
        assert err <= 0.02 * scale, (world, err, scale)
        top2 = ref_logits.topk(2, dim=-1).values
        margin = top2[..., 0] - top2[..., 1]
        agree = lg.argmax(-1) == ref_logits.argmax(-1)
        near_tie = margin < 2 * err + 1e-6
        # every disagreement is a near tie: TP sums f32 partials in another
        # order than TP=1's single GEMM. Exactness of the TP arithmetic itself
        # is pinned bitwise against the one-process emulation below
        # (test_tp_decode_bitwise_equals_emulation).
        assert bool((agree | near_tie).all()), (world, (~agree).sum().item(), err)
        # lock-step serving: same steps on every rank, no collective error
        lead = res[0]
        steps = {r["decode_steps"] for r in res}
        assert len(steps) == 1, f"ranks ran different step counts: {steps}"
        for r in res:
            assert not r["car_error"] and r["car_calls"] > 0 and r["car_fallbacks"] == 0
        for a, b in zip(lead["outs"], ref["outs"]):
            assert len(json.loads(a)["commands"]) == len(json.loads(b)["commands"])
        same = sum(a == b for a, b in zip(lead["outs"], ref["outs"]))
        print(f"TP={world}: logits max err {err:.3g} (scale {scale:.3g}), greedy agreement "
              f"{agree.float().mean().item():.3f}, identical outputs {same}/{len(ref['outs'])}")


def _failover_worker(rank, world, port, out_dir):
    """TP=2 on the shared GPU; rank 1 freezes mid-decode (SIGSTOP: a hung
    follower - its IPC memory stays mapped, so nothing reads freed memory).
    The leader's collectives time out, the error word rides on the step's
    sampled tokens (ERR_TOKEN), the group stops, and TPFailover swaps in a
    single-GPU engine."""
    import signal
    import threading
    import time
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    from loqa_hub_amd.engine.llm_engine import LLMEngine
    from loqa_hub_amd.models.configs import llama_config
    from loqa_hub_amd.models.llama import TPGroup
    from loqa_hub_amd.parallel.tp_control import TPControl
    from loqa_hub_amd.parallel.tp_serving import TPFailover
    cfg = llama_config("llama3-8b", n_layers=2)
    tp = TPGroup.create(rank, world, dist.group.WORLD, device=dev)   # runs the self-test
    eng = LLMEngine(cfg, dev, max_seqs=8, max_seq_len=512, tp=tp, seed=11)
    eng.tp_ctl = TPControl(rank, world, f"gpufo{port}", dist.group.WORLD)
    eng.tp_ctl.start_heartbeat(0.1)
    eng.warmup_graphs()
    if rank != 0:
        def freezer():
            while eng.stats.get("tp_records", 0) < 8:
                time.sleep(0.001)
            with open(os.path.join(out_dir, "frozen"), "w") as f:
                f.write(str(os.getpid()))
            os.kill(os.getpid(), signal.SIGSTOP)
        threading.Thread(target=freezer, daemon=True).start()
        eng.follow()
        os._exit(0)

    class Pipe:
        llm = eng

    class Proc:
        pipeline = Pipe()
        stats = {}
    proc = Proc()
    fo = TPFailover(proc, cfg, dev, seed=11, max_seqs=8, max_seq_len=512).attach(eng)
    res = {}
    t0 = time.monotonic()
    try:
        futs = [eng.submit_batch([r]) for r in _reqs(eng, 0)]
        res["outs"] = [r.output for f in futs for r in f.result(timeout=180)]
    except Exception as e:  # noqa: BLE001
        res["error"] = f"{type(e).__name__}: {e}"
    res["detect_s"] = time.monotonic() - t0
    res["car_error"] = tp.car.error()
    res["ready"] = fo.ready.wait(180)
    new = proc.pipeline.llm
    res["swapped"] = new is not eng and new.tp.world == 1
    if res["swapped"]:
        futs = [new.submit_batch([r]) for r in _reqs(new, 1)]
        res["fallback_outs"] = [r.output for f in futs for r in f.result(timeout=180)]
        new.stop()
    res["stats"] = dict(proc.stats)
    with open(os.path.join(out_dir, "failover.json"), "w") as f:
        json.dump(res, f)
    sys.stdout.flush()
    os._exit(0)


def test_tp_follower_hang_fails_over(tmp_path):
    """A TP follower that stops mid-decode: the leader fails its in-flight
    requests (no garbage tokens, no endless spin), stops the group and serves
    on the fallback engine with ``tp_degraded`` set."""
    import signal
    ctx = mp.get_context("spawn")
    port = _port()
    procs = [ctx.Process(target=_failover_worker, args=(r, 2, port, str(tmp_path)))
             for r in range(2)]
    for p in procs:
        p.start()
    procs[0].join(timeout=420)
    for p in procs:                     # the frozen follower, and anything left
        if p.is_alive():
            os.kill(p.pid, signal.SIGKILL)
            p.join(timeout=10)
    res = json.load(open(tmp_path / "failover.json"))
    print(res.get("error"), res["detect_s"], res["stats"])
    assert os.path.exists(tmp_path / "frozen")
    assert "error" in res and "CollectiveError" in res["error"], res
    assert res["car_error"]
    assert res["ready"] and res["swapped"]
    assert res["stats"]["tp_degraded"] == 1 and res["stats"]["tp_fallback_ready"] == 1
    assert len(res["fallback_outs"]) == 3
    for out, n in zip(res["fallback_outs"], (1, 3, 2)):
        assert len(json.loads(out)["commands"]) == n


def _decode_teacher(meta_fn, fwd_fn, add_seq, steps: int = 10):
    """Three sequences whose 24-token prompts go in through decode steps (8
    tokens per sequence per step, the jump-forward row limit of Llama-3-8B's
    GQA groups), then ``steps`` one-token steps of fixed tokens: the logits
    of every step (per shard) - no prefill kernel involved."""
    from loqa_hub_amd.engine.llm_engine import GenRequest
    reqs = [GenRequest(list(range(100 + 7 * i, 124 + 7 * i)), []) for i in range(3)]
    for sid, r in enumerate(reqs, start=1):
        r.seq_id = sid
        add_seq(sid)
    feeds_seq = [[r.prompt[c:c + 8] for r in reqs] for c in range(0, 24, 8)]
    feeds_seq += [[[(1000 + 37 * t + 11 * i) % 120000] for i in range(3)] for t in range(steps)]
    out = []
    for feeds in feeds_seq:
        T = sum(len(f) for f in feeds)
        meta = meta_fn(reqs, feeds, 3, 16 if T <= 16 else 32)
        out.append(fwd_fn(meta))
    torch.cuda.synchronize()
    return out


def _bitwise_worker(rank, world, port, out_dir, pro=0):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LOQA_NO_TUNE="1",
                      LOQA_TP_PROLOGUE=str(pro))
    if world >= 8:
        os.environ["GPU_MAX_HW_QUEUES"] = "1"
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        from loqa_hub_amd.engine.llm_engine import LLMEngine
        from loqa_hub_amd.models.configs import llama_config
        from loqa_hub_amd.models.llama import TPGroup
        cfg = llama_config("llama3-8b", n_layers=4)
        tp = TPGroup.create(rank, world, dist.group.WORLD, device=dev)
        eng = LLMEngine(cfg, dev, max_seqs=8, max_seq_len=512, tp=tp, seed=11, use_graphs=False)

        def meta_fn(reqs, feeds, B, T):
            max_q, max_ctx, host = eng._meta(reqs, feeds, True, B, T)
            return eng._build_meta(eng._to_device(host), max_q, max_ctx, True)

        def fwd(meta):
            lg = eng.model.forward_decode_fused(meta, eng.kv.k, eng.kv.v, eng.attn_ws, eng.scratch)[:3]
            lgf = lg.float().contiguous()
            tok = tp.car.argmax(lgf, lgf.argmax(1).to(torch.int32), rank * lgf.shape[1])
            return lgf.cpu(), tok.cpu()
        real = _decode_teacher(meta_fn, fwd, lambda sid: eng.kv.pool.add_seq(sid, []))
        torch.save({"logits": [l for l, _ in real], "tokens": [t for _, t in real]},
                   os.path.join(out_dir, f"real{world}_r{rank}.pt"))
        dist.barrier()
        if rank == 0:
            from loqa_hub_amd.parallel.tp_emulation import TPEmulation
            emu = TPEmulation(cfg, dev, world, seed=11, max_seqs=8, max_seq_len=512)

            def emeta(reqs, feeds, B, T):
                return emu.meta(reqs, feeds, B, T)[0]

            def efwd(meta):
                shards = [s[:3].float().contiguous() for s in emu.forward_decode_fused(meta)]
                tok = TPEmulation.argmax_combine([s.cpu() for s in shards],
                                                 [s.argmax(1).to(torch.int32).cpu() for s in shards])
                return [s.cpu() for s in shards], tok
            em = _decode_teacher(emeta, efwd, emu.add_seq)
            torch.save({"logits": [l for l, _ in em], "tokens": [t for _, t in em]},
                       os.path.join(out_dir, f"emu{world}.pt"))
        dist.barrier()
    finally:
        dist.destroy_process_group()
    sys.stdout.flush()
    os._exit(0)


@pytest.mark.parametrize("world,pro", [(2, 0), (4, 0), (8, 0), (8, 1)])
def test_tp_decode_bitwise_equals_emulation(tmp_path, world, pro):
    """TP=W over the real IPC collectives (W processes sharing cuda:0) vs the
    single-process TP emulation of the same W shards (parallel/tp_emulation.py):
    every logit shard of every decode step and every combined greedy token is
    BITWISE equal (replaces round 3's 2% / 90% tolerances). ``pro``: the step
    with the all-reduces as prologue items of the consuming GEMMs, the ranks'
    grids capped so they are resident together (CustomAllReduce.prologue_wgs)."""
    ctx = mp.get_context("spawn")
    port = _port()
    procs = [ctx.Process(target=_bitwise_worker, args=(r, world, port, str(tmp_path), pro))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=600)
    for p in procs:
        if p.is_alive():
            p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    emu = torch.load(tmp_path / f"emu{world}.pt", weights_only=True)
    for r in range(world):
        real = torch.load(tmp_path / f"real{world}_r{r}.pt", weights_only=True)
        for step, (a, b) in enumerate(zip(real["logits"], emu["logits"])):
            assert torch.equal(a, b[r]), (world, r, step, (a - b[r]).abs().max().item())
        for step, (a, b) in enumerate(zip(real["tokens"], emu["tokens"])):
            assert torch.equal(a.to(torch.int32), b.to(torch.int32)), (world, r, step, a, b)


def _solo_tp_engine(n_layers=3, world=8):
    """One TP rank of Llama-3-8B-shaped layers with one-rank collectives (the
    config-5 projection's setup, scripts/config5_projection.py)."""
    from loqa_hub_amd.engine.llm_engine import GenRequest, LLMEngine
    from loqa_hub_amd.models.configs import llama_config
    from loqa_hub_amd.models.llama import TPGroup
    from loqa_hub_amd.parallel.custom_allreduce import CustomAllReduce
    dev = torch.device("cuda", 0)
    cfg = llama_config("llama3-8b", n_layers=n_layers)
    tp = TPGroup(0, world, None, CustomAllReduce(solo=True))
    eng = LLMEngine(cfg, dev, max_seqs=8, max_seq_len=512, tp=tp, use_graphs=False, seed=5)
    reqs = []
    for i, ctx in enumerate([300, 17, 129, 64]):
        r = GenRequest(list(range(5 + i, 5 + i + ctx)), [])
        r.seq_id = eng._next_id
        eng._next_id += 1
        eng.kv.pool.add_seq(r.seq_id, [])
        eng._meta([r], [r.prompt], decode=False)
        reqs.append(r)
    return eng, reqs


@pytest.mark.parametrize("Mpad,per", [(16, 2), (32, 3)])
def test_tp_prologue_step_bitwise(Mpad, per):
    """The TP decode step with the all-reduces and the attention run as GEMM
    prologues (4 launches per layer, gemm_skinny.hip PRO) gives BITWISE the
    logits of the 7-launch step, eagerly and replayed from a HIP graph (the
    launches' ticket counters reset themselves)."""
    import numpy as np

    from loqa_hub_amd import ops
    eng, reqs = _solo_tp_engine()
    feeds = [[7 + j for j in range(per)] for _ in reqs]
    max_q, max_ctx, host = eng._meta(reqs, feeds, True, len(reqs), Mpad)
    host["mask_rows"] = np.zeros(len(reqs), np.int32)
    d = eng._to_device(host)
    meta = eng._build_meta(d, max_q, max_ctx, True)
    k0, v0 = eng.kv.k.clone(), eng.kv.v.clone()

    def step(pro: bool):
        old = ops.TP_PROLOGUE
        ops.TP_PROLOGUE = pro
        try:
            eng.kv.k.copy_(k0)
            eng.kv.v.copy_(v0)
            return eng.model.forward_decode_fused(meta, eng.kv.k, eng.kv.v, eng.attn_ws,
                                                  eng.scratch, 128).float().clone()
        finally:
            ops.TP_PROLOGUE = old
    ref_ = step(False)
    got = step(True)
    assert torch.equal(got, ref_), (got - ref_).abs().max().item()
    assert int(eng.scratch.pro_ctr.abs().sum()) == 0
    # graph capture + replays
    old = ops.TP_PROLOGUE
    ops.TP_PROLOGUE = True
    try:
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            step(True)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        eng.kv.k.copy_(k0)
        eng.kv.v.copy_(v0)
        with torch.cuda.graph(g):
            out = eng.model.forward_decode_fused(meta, eng.kv.k, eng.kv.v, eng.attn_ws, eng.scratch, 128)
        for _ in range(3):
            eng.kv.k.copy_(k0)
            eng.kv.v.copy_(v0)
            g.replay()
            torch.cuda.synchronize()
            assert torch.equal(out.float(), ref_)
    finally:
        ops.TP_PROLOGUE = old
