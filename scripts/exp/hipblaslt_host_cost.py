"""Host-side cost of a hipBLASLt GEMM call through torch (F.linear) for a NEW
row count each call (as prefill passes see: every prompt length differs) vs a
repeated one: if torch re-queries the algorithm heuristics per new shape, the
first call of a shape is far slower on the host. Prints JSON."""
import json
import time

import torch

dev = torch.device("cuda", 0)
w = torch.randn(6144, 4096, device=dev, dtype=torch.bfloat16)
xs = torch.randn(1024, 4096, device=dev, dtype=torch.bfloat16)
torch.nn.functional.linear(xs[:300], w)
torch.cuda.synchronize()


def host_us(M):
    t0 = time.perf_counter()
    torch.nn.functional.linear(xs[:M], w)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    return (t1 - t0) * 1e6


rep = [host_us(300) for _ in range(20)]
new = [host_us(M) for M in range(301, 341)]
again = [host_us(M) for M in range(301, 341)]
print(json.dumps({"repeat_M_median_us": sorted(rep)[10], "new_M_median_us": sorted(new)[20],
                  "second_visit_median_us": sorted(again)[20], "new_M_max_us": max(new)}))
