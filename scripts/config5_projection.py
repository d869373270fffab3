"""BASELINE config 5 (Llama-3-70B intent decoder at TP=8) projected from ONE
MI355X: time one TP rank's decode step at its real shard shapes.

The rank-0 shard of Llama-3-70B (qkv 8192 -> 1280, o 1024 -> 8192, gate|up
8192 -> 7168, down 3584 -> 8192, lm_head 8192 -> 16032; the d = 8192 decode
GEMMs tuned by the same contended tuner as serving) runs the fused TP decode
step - 80 layers x (qkv, attention, o -> residual all-reduce, gate|up, down ->
residual all-reduce), final norm, vocab-shard lm_head, argmax combine -
graph-captured and replayed. The collectives run the real custom all-reduce
kernels on a one-rank handle (``CustomAllReduce(solo=True)``): the same
reduce / statistics / argmax work over local buffers, without the cross-GPU
flag exchanges and xGMI reads. The projection adds those from a stated
per-collective model (``--xgmi-us``), so the result is a range, not a claim.

    python scripts/config5_projection.py [--batch 8] [--ctx 384] [--tokens 16]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-70b")
    ap.add_argument("--tp", type=int, default=8)
    ap.add_argument("--batch", type=int, default=8, help="live sequences per step")
    ap.add_argument("--tokens", type=int, default=16, help="padded token rows per step (Mpad)")
    ap.add_argument("--ctx", type=int, default=384, help="context length of every sequence")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--layers", type=int, default=0, help="override layer count (0: the model's)")
    ap.add_argument("--xgmi-us", default="3,6",
                    help="extra latency per cross-GPU collective (low,high): flag exchange + xGMI reads")
    ap.add_argument("--prefill-rows", type=int, default=320,
                    help="also time this rank's prompt pass over this many tokens (0: skip)")
    ap.add_argument("--xgmi-gbps", default="40,60",
                    help="effective GB/s per xGMI link (low,high) for the prompt pass's two-shot "
                         "all-reduces (7 links per GPU)")
    ap.add_argument("--steps-per-command", type=float, default=40.0,
                    help="decode steps per added command with 8 loaded streams (marginal ms / ms "
                         "per step of the 70B TP=1 8-stream run: profiles/config5_tp1_r2.json "
                         "1035.73 / 25.884 = 40; r5_config5_tp1.json 972.93 / 24.743 = 39.3)")
    ap.add_argument("--steps-per-command-1stream", type=float, default=None,
                    help="measured decode steps per added command of ONE stream (the reference's "
                         "scenario: one multi-command utterance; scripts/bench_configs.py --config 5 "
                         "--streams 1, decode_steps_per_added_command)")
    ap.add_argument("--stt-ms-per-command-1stream", type=float, default=0.0,
                    help="the STT phase's growth per added command of that run (a longer "
                         "transcript; independent of the LLM's TP degree)")
    a = ap.parse_args()
    from loqa_hub_amd.engine.llm_engine import GenRequest, LLMEngine
    from loqa_hub_amd.models.configs import llama_config
    from loqa_hub_amd.models.llama import TPGroup
    from loqa_hub_amd.parallel.custom_allreduce import CustomAllReduce

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cfg = llama_config(a.model, **({"n_layers": a.layers} if a.layers else {}))
    tp = TPGroup(0, a.tp, None, CustomAllReduce(solo=True))
    t0 = time.perf_counter()
    eng = LLMEngine(cfg, dev, max_seqs=max(8, a.batch), max_seq_len=max(512, a.ctx + 64), tp=tp,
                    use_graphs=False)
    t_init = time.perf_counter() - t0
    # B sequences with `ctx` tokens of context, each feeding T / B tokens
    per = max(1, a.tokens // a.batch)
    reqs = [GenRequest(list(range(5, 5 + a.ctx - per)), []) for _ in range(a.batch)]
    for r in reqs:
        r.seq_id = eng._next_id
        eng._next_id += 1
        eng.kv.pool.add_seq(r.seq_id, [])
        # claim the context's KV slots (contents do not matter for timing)
        eng._meta([r], [r.prompt], decode=False)
    feeds = [[7] * per for _ in reqs]
    max_q, max_ctx, host = eng._meta(reqs, feeds, True, a.batch, a.tokens)
    host["mask_rows"] = np.zeros(a.batch, np.int32)
    d = eng._to_device(host)
    meta = eng._build_meta(d, max_q, max_ctx, True)

    def step():
        logits = eng.model.forward_decode_fused(meta, eng.kv.k, eng.kv.v, eng.attn_ws, eng.scratch,
                                                eng.attn_split_keys)
        return eng._tp_argmax(logits[: a.batch], d["mask_rows"])

    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        for _ in range(2):
            step()
    torch.cuda.current_stream(dev).wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(a.iters):
        g.replay()
    ev1.record()
    torch.cuda.synchronize()
    step_ms = ev0.elapsed_time(ev1) / a.iters
    L = cfg.n_layers
    n_coll = 2 * L + 1
    lo, hi = (float(v) for v in a.xgmi_us.split(","))
    w = eng.weights
    # the bytes one fused decode step streams: the norm-folded / row-permuted
    # qkv and gate|up copies, o, down, the vocab-shard lm_head (decode_layers
    # also holds the unfused qkv / gate|up copies, which the step never reads)
    fused_keys = ("wqkv_f", "wo", "w_gate_up_f", "w_down")
    shard_bytes = sum(P[k].numel() * P[k].element_size() for P in w.decode_layers
                      for k in fused_keys) + w.lm_head_p.numel() * 2
    out = {"model": cfg.name, "tp": a.tp, "rank_shard_weight_GB": round(shard_bytes / 1e9, 2),
           "batch": a.batch, "token_rows": a.tokens, "ctx": a.ctx, "layers": L,
           "rank_step_ms_local_collectives": round(step_ms, 3),
           "rank_step_weight_TBps": round(shard_bytes / (step_ms * 1e-3) / 1e12, 2),
           "collectives_per_step": n_coll, "xgmi_us_per_collective": [lo, hi],
           "projected_step_ms": [round(step_ms + n_coll * lo / 1e3, 3),
                                 round(step_ms + n_coll * hi / 1e3, 3)],
           "init_s": round(t_init, 1)}
    spc = a.steps_per_command
    out["steps_per_added_command"] = spc
    out["projected_ms_per_added_command"] = [round(spc * v, 1) for v in out["projected_step_ms"]]
    out["reference_bar_ms_per_added_command"] = 200.0
    if a.steps_per_command_1stream:
        s1 = a.steps_per_command_1stream
        out["steps_per_added_command_1stream"] = s1
        out["stt_ms_per_added_command_1stream"] = a.stt_ms_per_command_1stream
        out["projected_ms_per_added_command_1stream"] = [
            round(s1 * v + a.stt_ms_per_command_1stream, 1) for v in out["projected_step_ms"]]
    if a.prefill_rows > 0 and "wqkv" in (w.layers[0] if w.layers else {}):
        # this rank's prompt pass (hand-written GEMMs on its shards; the
        # row-parallel partials' all-reduces are no-ops on the one-rank handle
        # and are modelled below: two-shot, 2 (W-1)/W of the tensor per rank
        # over 7 links)
        T = a.prefill_rows
        r = GenRequest(list(range(7, 7 + T)), [])
        r.seq_id = eng._next_id
        eng._next_id += 1
        eng.kv.pool.add_seq(r.seq_id, [])
        mq, mc, hp = eng._meta([r], [r.prompt], decode=False)
        dp = eng._to_device(hp)
        pm = eng._build_meta(dp, mq, mc, False)

        def pass_():
            return eng.model.logits(eng.model.forward(pm, eng.kv.k, eng.kv.v, eng.attn_ws))
        for _ in range(2):
            pass_()
        torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            pass_()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        pf_ms = sorted(ts)[len(ts) // 2]
        nbytes = T * cfg.d_model * 2
        per_rank = 2 * (a.tp - 1) / a.tp * nbytes
        glo, ghi = (float(v) for v in a.xgmi_gbps.split(","))
        n_ar = 2 * L
        ar = [n_ar * (per_rank / (7 * g * 1e9) * 1e3 + lo / 1e3) for g in (ghi, glo)]
        out["prefill"] = {"rows": T, "rank_pass_ms_local": round(pf_ms, 3),
                          "allreduces": n_ar, "allreduce_bytes": nbytes,
                          "projected_pass_ms": [round(pf_ms + ar[0], 2), round(pf_ms + ar[1], 2)],
                          "gemms": "ops.proj (gemm_sk / gemm_ws), no hipBLASLt"}
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
