import torch, sys
sys.path.insert(0, '.')
from loqa_hub_amd import ops
from loqa_hub_amd.ops import reference as ref
torch.manual_seed(5)
K=1024; N=512
for Mpad, xl, wr, rt in [(64,0,1,1),(64,0,4,1),(64,1,4,1),(128,1,4,1)]:
    x = torch.randn(Mpad, K).bfloat16()
    w = (torch.randn(N, K) * 0.03).bfloat16()
    tiles=4
    rs = (torch.rand(tiles*Mpad)*300+50)
    outs=[]
    for dev in ("cpu","cuda"):
        wp = ops.shuffle_weight(w.to(dev)); scr = ops.FusedScratch(dev)
        scr.rowsq[:tiles*Mpad].copy_(rs.to(dev))
        y = ops.skinny_fused(x.to(dev), wp, "act", scr, splits=1, wr=wr, rt=rt, xl=xl, norm="rms", rowsq_tiles=tiles)
        outs.append(y.float().cpu())
    a,b=outs
    rel=float((b-a).norm()/a.norm())
    # per-row error
    rr=((b-a).norm(dim=1)/a.norm(dim=1))
    print(Mpad, xl, wr, rt, "rel", rel, "bad rows", (rr>0.02).nonzero().flatten().tolist()[:20], "ratio row0", float(b[0].norm()/a[0].norm()))
