"""Grid-barrier cost on this chip: 256 barriers per launch with G workgroups,
alone and beside the Llama gate|up weight stream (the megakernel feasibility
question for the Whisper decoder)."""
import ctypes, json, os, sys, threading, time
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from loqa_hub_amd import ops  # noqa: E402
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libgemv_exp.so"))
vp, ci, cu = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint
lib.exp_barrier.argtypes = [vp, cu, ci, vp, vp, ci, vp]
dev = torch.device("cuda", 0)
ctr = torch.zeros(1, dtype=torch.int32, device=dev)
buf = torch.zeros(4096, device=dev)
err = torch.zeros(1, dtype=torch.int32, device=dev)
base = [0]


def run(G, phases=256):
    st = torch.cuda.current_stream().cuda_stream
    lib.exp_barrier(ctr.data_ptr(), base[0] & 0xffffffff, phases, buf.data_ptr(), err.data_ptr(), G, st)
    base[0] += phases * G


def timed(G, n=10):
    run(G)
    torch.cuda.synchronize()
    ts = []
    for _ in range(n):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); run(G); b.record(); b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / 256)
    ts.sort()
    return ts[len(ts) // 2]


bf = dict(dtype=torch.bfloat16, device=dev)
ws = [ops.shuffle_weight(torch.randn(28672, 4096, **bf) * 0.02) for _ in range(3)]
x = torch.randn(16, 4096, **bf)
scr = ops.FusedScratch(dev)
scr.rowsq[: 128 * 16].fill_(32.0)
stop = threading.Event()


def bg():
    torch.cuda.set_device(dev)
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        i = 0
        while not stop.is_set():
            for _ in range(8):
                ops.skinny_fused(x, ws[i % 3], "silu", scr, splits=1, rt=2, wr=4, norm=True, rowsq_tiles=128)
                i += 1
            s.synchronize()


torch.cuda.set_stream(torch.cuda.Stream(dev))
res = {}
for G in (32, 64, 80, 128, 256):
    res[f"alone_G{G}_us_per_barrier"] = round(timed(G), 3)
th = threading.Thread(target=bg, daemon=True)
th.start()
time.sleep(0.5)
for G in (32, 64, 80, 128):
    res[f"beside_gateup_G{G}_us_per_barrier"] = round(timed(G), 3)
stop.set()
th.join()
res["err"] = int(err.item())
print(json.dumps(res), flush=True)
