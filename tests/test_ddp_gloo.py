"""CPU, world_size 2 over gloo: the data-parallel gradient reducer and the buffer
broadcast (the N>1 path of bench.py / train_enhanced.main)."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from superresolution_for_pdes_amd.distributed import GradReducer, DataParallel, shard_indices
        n = 1000
        flat = torch.arange(n, dtype=torch.float32) * (rank + 1)
        red = GradReducer(bucket_bytes=256 * 4)
        red.begin(flat)
        for upto in (100, 300, 301, 800):     # growing finished prefix, as the executor reports it
            red.ready(upto)
        red.finish()
        want = torch.arange(n, dtype=torch.float32) * (sum(r + 1 for r in range(world)) / world)
        ok_grad = torch.allclose(flat, want)
        nb = red.n_buckets

        class Tiny(torch.nn.Module):
            def __init__(self):
                super().__init__()
                self.lin = torch.nn.Linear(3, 2)
                self.bn = torch.nn.BatchNorm1d(2)

            def forward(self, x):
                return self.bn(self.lin(x))

        torch.manual_seed(rank)                # different init per rank
        t = Tiny()
        with torch.no_grad():
            t.bn.running_mean.fill_(float(rank + 1))
        dp = DataParallel(t)
        w0 = t.lin.weight.detach().clone()
        dist.broadcast(w0, 0)
        ok_params = torch.equal(t.lin.weight.detach(), w0)
        ok_buf = torch.equal(t.bn.running_mean, torch.ones(2))
        dp.train()
        dp(torch.randn(4, 3))
        idx = shard_indices(10, rank, world, seed=3)
        q.put((rank, ok_grad, nb, ok_params, ok_buf, idx.tolist()))
    finally:
        dist.destroy_process_group()


def test_grad_reducer_and_buffer_broadcast_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    for rank, ok_grad, nb, ok_params, ok_buf, _ in res:
        assert ok_grad, rank
        assert nb == 4, nb          # 3 full 256-element buckets + the tail
        assert ok_params and ok_buf
    shards = [set(r[5]) for r in res]
    assert not shards[0] & shards[1] and shards[0] | shards[1] == set(range(10))
