"""Prefill GEMMs at M ~ 318: hipBLASLt picks few output tiles for N = 4096
(o, down). Split-K through one strided-batched GEMM + a sum, vs plain linear."""
import json
import torch
dev = torch.device("cuda")
out = {}
for name, (N, K) in {"o": (4096, 4096), "down": (4096, 14336), "qkv": (6144, 4096),
                     "gate_up": (28672, 4096)}.items():
    ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(4)]
    for M in (318, 636):
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        ref = (x.float() @ ws[0].float().t())
        def plain(i):
            return torch.nn.functional.linear(x, ws[i])
        def splitk(i, S):
            xs = x.view(M, S, K // S).transpose(0, 1)                 # [S, M, K/S]
            wv = ws[i].view(N, S, K // S).permute(1, 2, 0)            # [S, K/S, N]
            part = torch.bmm(xs, wv, out_dtype=torch.float32) if hasattr(torch, "bmm") else None
            return part.sum(0).to(torch.bfloat16)
        def timeit(fn):
            for i in range(4):
                fn(i)
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for i in range(40):
                fn(i % 4)
            b.record()
            torch.cuda.synchronize()
            return round(a.elapsed_time(b) / 40 * 1e3, 1)
        out[f"{name}:M{M}:plain"] = timeit(plain)
        for S in (2, 4, 8):
            try:
                err = float((splitk(0, S).float() - ref).norm() / ref.norm())
                out[f"{name}:M{M}:S{S}"] = [timeit(lambda i: splitk(i, S)), round(err, 5)]
            except Exception as e:  # noqa: BLE001
                out[f"{name}:M{M}:S{S}"] = str(e)[:80]
    del ws
print(json.dumps(out))
