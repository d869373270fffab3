"""Tiled MFMA GEMM (csrc/kernels/gemm_tile.hip) vs hipBLASLt (torch linear) on
the encoder / conv stem / cross-K/V / prefill shapes. Weights rotate over
enough copies to exceed the 256 MiB Infinity Cache where a real pass reads
them cold. Prints one JSON line per (shape, variant): median us per call."""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from loqa_hub_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(0)
LAYOUTS = [int(v) for v in os.environ.get("GT_LAYOUTS", "0,1,2,3,4,5,6,7,8,9").split(",")]


def timeit(fn, iters=20, reps=5):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(iters):
            fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / iters)
    ts.sort()
    return ts[len(ts) // 2]


def weights(N, K, cold=True):
    n = max(1, min(16, (512 << 20) // (N * K * 2))) if cold else 1
    return [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.05 for _ in range(n)]


def run(name, M, N, K, epi="bf16", bias=False, act=None, splits=(1,), conv=None):
    if conv is not None:
        B, stride, cin = conv
        tin = (M // B - 1) * stride + 1 if stride == 1 else (M // B) * stride
        x = torch.randn(B * tin, cin, device=dev, dtype=torch.bfloat16)
    else:
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    ws = weights(N, K)
    b = torch.randn(N, device=dev, dtype=torch.float32) * 0.1 if bias else None
    flop = 2.0 * M * N * K
    it = [0]

    def nxt():
        it[0] = (it[0] + 1) % len(ws)
        return ws[it[0]]

    # hipBLASLt reference (the path this kernel replaces)
    if conv is None:
        bb = b.to(torch.bfloat16) if b is not None else None
        if epi == "swiglu":
            def hb():
                y = torch.nn.functional.linear(x, nxt())
                return ops.silu_mul(y) if False else y
        else:
            def hb():
                return torch.nn.functional.linear(x, nxt(), bb)
    else:
        B, stride, cin = conv
        def hb():
            cols = ops.conv_k3_im2col_ref(x, B, x.shape[0] // B, stride)
            return torch.nn.functional.linear(cols, nxt())
    us = timeit(hb)
    print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "impl": "hipblaslt", "us": round(us, 2),
                      "tflops": round(flop / us / 1e6, 1)}), flush=True)
    # correctness vs fp32 once
    w0 = ws[0]
    for lay in LAYOUTS:
        for S in splits:
            e = epi if S == 1 else "slabs"
            try:
                y = ops.gemm_tile(x, w0, bias=b if e != "slabs" else None, act=act, epi=e, splits=S,
                                  layout=lay, conv=(conv[0], conv[1]) if conv else None)
                xr = ops.conv_k3_im2col_ref(x, conv[0], x.shape[0] // conv[0], conv[1]) if conv else x
                r = ops._gt_ref(xr.cpu(), w0.cpu(), b.cpu() if (b is not None and e != "slabs") else None,
                                act, None, e, S)
                err = (y.float().cpu() - r.float()).abs().max().item() / max(r.float().abs().max().item(), 1e-6)
                us = timeit(lambda: ops.gemm_tile(x, nxt(), bias=b if e != "slabs" else None, act=act,
                                                  epi=e, splits=S, layout=lay,
                                                  conv=(conv[0], conv[1]) if conv else None))
                print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "impl": f"tile{lay}", "S": S,
                                  "us": round(us, 2), "tflops": round(flop / us / 1e6, 1),
                                  "rel_err": round(err, 5)}), flush=True)
            except Exception as ex:  # noqa: BLE001
                print(json.dumps({"shape": name, "impl": f"tile{lay}", "S": S, "error": str(ex)[:200]}),
                      flush=True)


SHAPES = os.environ.get("GT_SHAPES", "all")
if SHAPES in ("all", "enc"):
    run("enc_qkv_b1", 1500, 3840, 1280, bias=True)
    run("enc_fc1_b1", 1500, 5120, 1280, bias=True, act="gelu")
    run("enc_fc2_b1", 1500, 1280, 5120, bias=True, splits=(1, 2, 4))
    run("enc_qkv_b2", 3000, 3840, 1280, bias=True)
    run("enc_fc2_b2", 3000, 1280, 5120, bias=True, splits=(1, 2))
    run("xkv_all_b1", 1500, 81920, 1280)
    run("conv1_b1", 3000, 1280, 384, conv=(1, 1, 128), bias=True, act="gelu")
    run("conv2_b1", 1500, 1280, 3840, conv=(1, 2, 1280), bias=True, act="gelu")
if SHAPES in ("all", "llm"):
    run("llm_qkv_318", 318, 6144, 4096, splits=(1, 2))
    run("llm_gu_318", 318, 28672, 4096, epi="swiglu")
    run("llm_qkv_600", 600, 6144, 4096, splits=(1, 2))
    run("llm_gu_600", 600, 28672, 4096, epi="swiglu")
