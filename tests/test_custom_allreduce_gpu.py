"""Custom IPC one-shot / two-shot all-reduce (K17). The round-end box has one GPU, so the
ranks share cuda:0: the IPC mapping, the signal protocol, the epoch double
buffering and graph replay are exercised; the cross-GPU xGMI reads are the
same code path with different physical links. Handles are exchanged over gloo."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        from loqa_hub_amd.parallel.custom_allreduce import CustomAllReduce
        car = CustomAllReduce(dist.group.WORLD, slot_bytes=4 << 20)
        ok = True
        # one-shot (small, decode) and two-shot (>= 512 KB, prefill) sizes
        for dt, n in ((torch.bfloat16, 16 * 8192), (torch.float32, 16 * 4096), (torch.bfloat16, 8),
                      (torch.bfloat16, 1 << 20), (torch.float32, 3 << 18)):
            xs = [torch.randn(n, generator=torch.Generator().manual_seed(100 * r + n)).to(dt)
                  for r in range(world)]
            expect = torch.zeros(n)
            for x in xs:
                expect += x.float()
            x = xs[rank].cuda()
            car(x)
            torch.cuda.synchronize()
            ok &= bool(torch.allclose(x.float().cpu(), expect.to(dt).float(), atol=2e-2, rtol=2e-2))
        # graph capture: the epoch lives on the device, so replays stay in step
        x = torch.full((4096,), float(rank + 1), device="cuda", dtype=torch.bfloat16)
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            with torch.cuda.graph(g):
                car(x)
                car(x)
        for _ in range(3):
            x.fill_(float(rank + 1))
            g.replay()
        torch.cuda.synchronize()
        tot = world * (world + 1) / 2
        ok &= bool((x.float() == tot * world).all().item())
        ok &= not car.error() and car.fallbacks == 0
        # ineligible tensors (here: host memory) take the process-group fallback
        host = torch.ones(16)
        car(host)
        ok &= bool((host == world).all().item()) and car.fallbacks == 1
        car.close()
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_custom_allreduce_single_gpu(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    alive = [p for p in procs if p.is_alive()]
    for p in alive:
        p.kill()
    assert not alive, "custom all-reduce ranks hung"
    res = dict(q.get(timeout=5) for _ in range(world))
    assert all(res.values()), res

