"""Llama-3-8B decode GEMMs at Mpad 16 in isolation (graph-replayed, cold
weights cycled over enough copies to outgrow the Infinity Cache): the fused
qkv with its RMSNorm prologue + RoPE / paged-KV epilogue against the same
weights and layout with the plain "act" epilogue and no norm, per layout, and
the o / down / gate|up kernels for the per-byte rate. Prints JSON lines."""
import copy
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from loqa_hub_amd import ops  # noqa: E402
from loqa_hub_amd.ops import reference as ref  # noqa: E402

dev = torch.device("cuda", 0)
bf = dict(dtype=torch.bfloat16, device=dev)
torch.manual_seed(0)
H, Hkv, D, d = 32, 8, 128, 4096
Mpad = 16
scr = ops.FusedScratch(dev)


def copies_of(lin, nbytes):
    out = [lin]
    for _ in range(min(15, -(-(768 << 20) // nbytes) - 1)):
        c = copy.copy(lin)
        c.wp = lin.wp.clone()
        out.append(c)
    return out


def bench(name, lin, mode, cfgs, nbytes, **kw):
    cs = copies_of(lin, nbytes)
    it = [0]
    x = torch.randn(Mpad, lin.K, **bf)
    for (S, rt, wr) in cfgs:
        def run():
            it[0] = (it[0] + 1) % len(cs)
            ops.skinny_fused(x, cs[it[0]], mode, scr, splits=S, rt=rt, wr=wr, **kw)
        try:
            ms = ops.graph_time(run, reps=2 * len(cs))
            us = ms * 1e3 / (2 * len(cs))
            print(json.dumps({"kernel": name, "mode": mode, "S": S, "rt": rt, "wr": wr,
                              "us": round(us, 2), "TBps": round(nbytes / us / 1e6, 2)}), flush=True)
        except Exception as e:  # noqa: BLE001
            print(json.dumps({"kernel": name, "S": S, "rt": rt, "wr": wr, "error": str(e)[:120]}))


wqkv = torch.randn((H + 2 * Hkv) * D, d, **bf) * 0.02
perm = ref.perm_rope_qkv(H, Hkv, D).to(dev)
norm_w = torch.ones(d, **bf)
qkv_rope = ops.FusedLinear(wqkv, norm="rms", norm_w=norm_w, perm=perm)
qkv_plain = ops.FusedLinear(wqkv)
nb = wqkv.numel() * 2
tiles = d // 32
scr.rowsq[: tiles * Mpad].fill_(float(d) / tiles)
kc = torch.zeros(8, Hkv, 16, D, **bf)
pos = torch.arange(Mpad, dtype=torch.int32, device=dev)
cfgs = [(1, 2, 1), (1, 1, 1), (2, 2, 1), (1, 1, 4), (1, 2, 4), (2, 1, 1)]
bench("qkv", qkv_rope, "rope", cfgs, nb, rowsq_tiles=tiles, positions=pos, cos_sin=None,
      q_out=torch.empty(Mpad, H * D, **bf), k_cache=kc, v_cache=torch.zeros_like(kc), slots=pos,
      n_heads=H, n_kv=Hkv, head_dim=D)
bench("qkv_plain_act", qkv_plain, "act", cfgs, nb)
wo = torch.randn(d, d, **bf) * 0.02
bench("o", ops.FusedLinear(wo), "resid", [(1, 1, 1), (1, 2, 1), (2, 2, 1), (2, 1, 1)], wo.numel() * 2,
      residual=torch.zeros(Mpad, d, **bf))
wd = torch.randn(d, 14336, **bf) * 0.02
bench("down", ops.FusedLinear(wd), "resid", [(2, 2, 1), (1, 2, 1), (4, 2, 1)], wd.numel() * 2,
      residual=torch.zeros(Mpad, d, **bf))
