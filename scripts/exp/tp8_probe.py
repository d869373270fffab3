#!/usr/bin/env python3
"""TP=N ranks sharing cuda:0: phase timings of the TP serving mechanics
(init, teacher-forced step, graph warm-up, served decode) with Llama-3-70B
shapes and a few layers, to locate where a full --config 5 --tp 8 rehearsal
spends its time. Every rank dumps its Python stacks if a phase stalls.

  python scripts/exp/tp8_probe.py --world 8 --layers 4 [--hwq 2]
"""
from __future__ import annotations

import argparse
import faulthandler
import json
import os
import socket
import sys
import time

import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def _worker(rank, world, port, args):
    if args.hwq:
        os.environ["GPU_MAX_HW_QUEUES"] = str(args.hwq)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LOQA_NO_TUNE="1")
    faulthandler.dump_traceback_later(args.stall, repeat=True)
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    t0 = time.perf_counter()

    def mark(what):
        if rank == 0:
            print(f"[{time.perf_counter() - t0:7.1f}s] {what}", flush=True)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    from loqa_hub_amd.engine.llm_engine import LLMEngine
    from loqa_hub_amd.engine.synthetic import make_batch
    from loqa_hub_amd.models.configs import llama_config
    from loqa_hub_amd.models.llama import TPGroup
    from loqa_hub_amd.parallel.tp_control import TPControl
    cfg = llama_config(args.model, n_layers=args.layers)
    tp = TPGroup.create(rank, world, dist.group.WORLD, device=dev)
    mark("tp group")
    eng = LLMEngine(cfg, dev, max_seqs=8, max_seq_len=512, tp=tp, seed=3, compact=args.compact)
    torch.cuda.synchronize()
    mark(f"engine ({torch.cuda.memory_allocated() / 2**30:.1f} GiB this rank)")
    eng.tp_ctl = TPControl(rank, world, f"probe{port}", dist.group.WORLD)
    n = eng.warmup_graphs()
    torch.cuda.synchronize()
    mark(f"warmup_graphs: {n} graphs")
    if rank == 0:
        from loqa_hub_amd.engine.grammar import multi_command_schema
        from loqa_hub_amd.engine.llm_engine import GenRequest
        from loqa_hub_amd.llm.prompts import build_multi_command_prompt
        utts = make_batch(0, 8, [1, 2, 3])
        s0 = eng.stats["decode_steps"]
        t1 = time.perf_counter()
        futs = [eng.submit_batch([GenRequest(eng.tok.encode(build_multi_command_prompt(u.text), bos=True),
                                             multi_command_schema(u.n_commands, min_response_tokens=8))])
                for u in utts[: args.reqs]]
        outs = [r.output for f in futs for r in f.result(timeout=args.serve_timeout)]
        dt = time.perf_counter() - t1
        steps = eng.stats["decode_steps"] - s0
        mark(f"served {len(outs)} requests: {steps} decode steps in {dt:.2f}s "
             f"({dt / max(1, steps) * 1e3:.1f} ms/step incl. prefill)")
        print(json.dumps({"world": world, "layers": args.layers, "steps": steps,
                          "ms_per_step": round(dt / max(1, steps) * 1e3, 2),
                          "car_calls": tp.car.calls if tp.car else None,
                          "car_error": bool(tp.car.error()) if tp.car else None}), flush=True)
        eng.stop()
    else:
        eng.follow()
    torch.cuda.synchronize()
    eng.tp_ctl.close()
    faulthandler.cancel_dump_traceback_later()
    dist.destroy_process_group()
    os._exit(0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--layers", type=int, default=4)
    ap.add_argument("--model", default="llama3-70b")
    ap.add_argument("--hwq", type=int, default=0, help="GPU_MAX_HW_QUEUES per rank (0: default)")
    ap.add_argument("--reqs", type=int, default=4)
    ap.add_argument("--compact", action="store_true")
    ap.add_argument("--stall", type=float, default=120.0)
    ap.add_argument("--serve-timeout", type=float, default=240.0)
    args = ap.parse_args()
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    mp.start_processes(_worker, args=(args.world, port, args), nprocs=args.world, join=True,
                       start_method="spawn")


if __name__ == "__main__":
    main()
