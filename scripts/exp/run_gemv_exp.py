import ctypes, json, os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libgemv_exp.so"))
vp, ci, cl = ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong
lib.exp_gemv.argtypes = [vp, vp, vp, ci, ci, ci, ci, ci, ci, ci, vp]
lib.exp_stream_read.argtypes = [vp, cl, vp, ci, vp]
lib.exp_gemv2.argtypes = [vp, vp, vp, ci, ci, ci, ci, ci, ci, ci, ci, vp]
MODE = sys.argv[1] if len(sys.argv) > 1 else "all"
dev = torch.device("cuda")
out = torch.zeros(1 << 20, device=dev)


def gtime(fns, reps=10):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for f in fns[:3]:
            f()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for f in fns:
            f()
    g.replay(); torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); g.replay(); b.record(); torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / len(fns))
    ts.sort()
    return ts[len(ts) // 2]


if MODE == "all":
  buf = torch.ones(1 << 30, device=dev, dtype=torch.bfloat16)
  for grid in (256, 512, 1024, 2048, 4096, 8192):
    t = gtime([lambda: lib.exp_stream_read(buf.data_ptr(), buf.numel() * 2, out.data_ptr(), grid,
                                           torch.cuda.current_stream().cuda_stream)] * 4)
    print(json.dumps({"exp": "stream_read_2GB", "grid": grid, "us": round(t, 1),
                      "TBps": round(buf.numel() * 2 / t / 1e6, 3)}), flush=True)
  del buf
for name, N, K in (("gate_up", 28672, 4096), ("down", 4096, 14336), ("qkv", 6144, 4096)):
    ncopy = max(2, -(-(1 << 30) // (N * K * 2)))
    ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) for _ in range(ncopy)]
    x = torch.randn(16, K, device=dev, dtype=torch.bfloat16)
    gb = N * K * 2 / 1e9
    for wr, wk, rt, u in ((1, 4, 1, 4), (1, 4, 2, 4), (1, 4, 2, 2), (1, 4, 4, 2), (4, 1, 1, 4), (4, 1, 1, 8),
                          (4, 1, 2, 4), (4, 2, 1, 4), (4, 2, 1, 8), (2, 2, 1, 4), (2, 2, 2, 4), (8, 1, 1, 4),
                          (4, 4, 1, 4), (1, 8, 1, 4), (1, 8, 2, 4)):
        for S in (1, 2, 4):
            for xf in (0, 1):
                def mk2(w):
                    return lambda: lib.exp_gemv2(x.data_ptr(), w.data_ptr(), out.data_ptr(), N, K, S, wr, wk,
                                                 rt, u, xf, torch.cuda.current_stream().cuda_stream)
                if mk2(ws[0])():
                    continue
                t = gtime([mk2(w) for w in ws] * 2)
                print(json.dumps({"exp": "gemv2", "shape": name, "wr": wr, "wk": wk, "rt": rt, "u": u, "S": S,
                                  "xf": xf, "us": round(t, 2), "TBps": round(gb / t * 1e3, 3)}), flush=True)
    for rt in ((1, 2, 4) if MODE == "all" else ()):
        for u in (2, 4, 8):
            for S in (1, 2, 4):
                for v, stag in ((0, 0), (1, 0), (2, 0), (3, 0), (0, 1), (2, 1)):
                    if N % (16 * rt) or K % (S * 128 * u):
                        continue
                    def mk(w):
                        return lambda: lib.exp_gemv(x.data_ptr(), w.data_ptr(), out.data_ptr(), N, K, S, rt, u,
                                                    v, stag, torch.cuda.current_stream().cuda_stream)
                    rc = mk(ws[0])()
                    if rc:
                        continue
                    t = gtime([mk(w) for w in ws] * 2)
                    print(json.dumps({"exp": "gemv", "shape": name, "rt": rt, "u": u, "S": S, "v": v,
                                      "stag": stag, "us": round(t, 2), "TBps": round(gb / t * 1e3, 3)}),
                          flush=True)
    del ws
