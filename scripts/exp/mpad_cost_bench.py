"""Llama-3-8B decode GEMMs at Mpad 16 vs 32 (isolated, graph-replayed, cold
weights): where does a 32-row decode step's extra cost come from? Every
(split-K, rows, waves-along-rows) layout under the 256-workgroup cap per
kernel; JSON lines."""
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
H, Hkv, D, d, F = 32, 8, 128, 4096, 14336
scr = ops.FusedScratch(dev)


def copies_of(lin, nbytes):
    out = [lin]
    for _ in range(min(15, -(-(768 << 20) // nbytes) - 1)):
        c = copy.copy(lin)
        c.wp = lin.wp.clone()
        out.append(c)
    return out


def bench(name, lin, mode, nbytes, mk_kw):
    cs = copies_of(lin, nbytes)
    N = lin.wp.shape[0] * 16
    for Mpad in (16, 32):
        x = torch.randn(Mpad, lin.K, **bf)
        kw = mk_kw(Mpad)
        for S in (1, 2, 4):
            for rt in (1, 2):
                for wr in (1, 4):
                    if wr == 4 and (N % (64 * rt) or (S != 1 and Mpad != 32)):
                        continue
                    if (N // (16 * rt * wr)) * S > 256 or lin.K % (S * 128):
                        continue
                    it = [0]
                    for xl in ((0, 1) if (Mpad == 32 and wr == 4 and N % (64 * rt) == 0) else (0,)):
                        def run():
                            it[0] = (it[0] + 1) % len(cs)
                            ops.skinny_fused(x, cs[it[0]], mode, scr, splits=S, rt=rt, wr=wr, xl=xl,
                                             **kw)
                        try:
                            us = ops.graph_time(run, reps=2 * len(cs)) * 1e3 / (2 * len(cs))
                            print(json.dumps({"kernel": name, "Mpad": Mpad, "S": S, "rt": rt, "wr": wr,
                                              "xl": xl, "us": round(us, 2),
                                              "TBps": round(nbytes / us / 1e6, 2)}), flush=True)
                        except Exception as e:  # noqa: BLE001
                            print(json.dumps({"kernel": name, "Mpad": Mpad, "S": S, "rt": rt, "wr": wr,
                                              "xl": xl, "error": str(e)[:100]}), flush=True)


def norm_kw(Mpad, extra=None):
    tiles = d // 32
    scr.rowsq[: tiles * Mpad].fill_(float(d) / tiles)
    kw = dict(rowsq_tiles=tiles)
    kw.update(extra or {})
    return kw


wgu = torch.randn(2 * F, d, **bf) * 0.02
gu = ops.FusedLinear(wgu, norm="rms", norm_w=torch.ones(d, **bf), perm=ref.perm_gate_up(F).to(dev))
bench("gate_up", gu, "silu", wgu.numel() * 2, lambda M: norm_kw(M))
del wgu, gu
wd = torch.randn(d, F, **bf) * 0.02
bench("down", ops.FusedLinear(wd), "resid", wd.numel() * 2,
      lambda M: dict(residual=torch.zeros(M, d, **bf)))
del wd
wqkv = torch.randn((H + 2 * Hkv) * D, d, **bf) * 0.02
qkv = ops.FusedLinear(wqkv, norm="rms", norm_w=torch.ones(d, **bf), perm=ref.perm_rope_qkv(H, Hkv, D).to(dev))
kc = torch.zeros(8, Hkv, 16, D, **bf)


def qkv_kw(M):
    pos = torch.arange(M, dtype=torch.int32, device=dev)
    return norm_kw(M, dict(positions=pos, cos_sin=None, q_out=torch.empty(M, H * D, **bf),
                           k_cache=kc, v_cache=torch.zeros_like(kc), slots=pos, n_heads=H, n_kv=Hkv,
                           head_dim=D))


bench("qkv", qkv, "rope", wqkv.numel() * 2, qkv_kw)
wo = torch.randn(d, d, **bf) * 0.02
bench("o", ops.FusedLinear(wo), "resid", wo.numel() * 2, lambda M: dict(residual=torch.zeros(M, d, **bf)))
