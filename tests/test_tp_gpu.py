"""Tensor-parallel serving on the GPU (BASELINE config 5's layout).

The round-end box has one MI355X, so the TP ranks share cuda:0 (as in
test_custom_allreduce_gpu.py): every collective is the real custom IPC kernel
(row-parallel residual all-reduce, vocab-parallel argmax combine), the decode
steps are captured HIP graphs replayed in lock step, and the scheduler of every
follower replays the leader's arrivals from the shared-memory control ring. Only
the physical links differ from an 8-GPU node.

Checks: TP=2 and TP=4 of Llama-3-8B's shapes (4 layers, to keep the test short)
produce token-identical constrained output to TP=1 on the same seed."""
import json
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


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
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
    for o in ref["outs"]:
        json.loads(o)
    for world in (2, 4):
        res = _run(world, str(tmp_path))
        lead = res[0]
        assert lead["outs"] == ref["outs"], (world, lead["outs"], ref["outs"])
        steps = {r["decode_steps"] for r in res}
        assert len(steps) == 1, f"ranks ran different step counts: {steps}"
        for r in res:
            assert not r["car_error"] and r["car_calls"] > 0 and r["car_fallbacks"] == 0
