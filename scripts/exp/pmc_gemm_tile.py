"""Short workload for rocprofv3 --pmc passes over the LDS-tiled MFMA GEMM
(csrc/kernels/gemm_tile.hip) on its serving shapes: the Whisper-large-v3
conv stem (implicit im2col, conv1 / conv2), the encoder fc2 as split-K slabs,
and the cross-attention K|V of all 32 decoder layers in one launch. Each
shape runs 8 times; scripts/pmc_summary.py reduces the counters."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from loqa_hub_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
bf = dict(dtype=torch.bfloat16, device=dev)
torch.manual_seed(0)
R = 8
d = 1280
mel = torch.randn(3000, 128, **bf)
w1 = torch.randn(d, 384, **bf) * 0.05
b1 = torch.zeros(d, device=dev)
x1 = torch.randn(3000, d, **bf)
w2 = torch.randn(d, 3 * d, **bf) * 0.02
pos = torch.randn(1500, d, **bf)
m = torch.randn(1500, 4 * d, **bf)
wfc2 = torch.randn(d, 4 * d, **bf) * 0.02
enc = torch.randn(1500, d, **bf)
wkv = torch.randn(32 * 2 * d, d, **bf) * 0.02
bkv = torch.zeros(32 * 2 * d, device=dev)
for _ in range(R):
    ops.gemm_tile(mel, w1, bias=b1, act="gelu", conv=(1, 1), layout=0)
    ops.gemm_tile(x1, w2, bias=b1, act="gelu", pos=pos, conv=(1, 2), layout=0)
    ops.gemm_tile(m, wfc2, epi="slabs", splits=4, layout=0)
    ops.gemm_tile(enc, wkv, bias=bkv, layout=7)
torch.cuda.synchronize()
