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


def _unet_layout_worker(rank, world, port, q):
    """GradReducer over the U-Net's REAL flat layout, fed the executor's group-end prefix sequence
    (unet_exec.FLAT_GROUPS order, _group_end_offsets), with different gradients per rank."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from superresolution_for_pdes_amd.distributed import GradReducer
        from superresolution_for_pdes_amd.models import UNet
        from superresolution_for_pdes_amd.unet_exec import FLAT_GROUPS, _group_end_offsets, flat_layout
        m = UNet()
        layout = flat_layout(m)
        total = layout[-1][2] + layout[-1][3]
        ends = _group_end_offsets(layout)
        g = torch.Generator().manual_seed(100 + rank)
        local = torch.randn(total, generator=g)
        flat = local.clone()
        bucket = 2 << 20                               # 2 MB = 524,288 floats
        red = GradReducer(bucket_bytes=bucket)
        red.begin(flat)
        tail_ok = True
        prev = 0
        for grp in FLAT_GROUPS:                        # the order the backward finishes groups
            assert ends[grp] >= prev                   # a growing prefix
            prev = ends[grp]
            red.ready(ends[grp])
            # nothing beyond the launched prefix is touched before finish()
            tail_ok &= torch.equal(flat[red.launched:], local[red.launched:])
        launched_before_finish = red.launched
        red.finish()
        # AVG semantics, checked here (a 31 MB tensor through the queue races the worker's exit)
        others = [torch.randn(total, generator=torch.Generator().manual_seed(100 + r)) for r in range(world)]
        avg_ok = torch.allclose(flat, sum(others) / world, rtol=0, atol=1e-6)
        q.put((rank, total, avg_ok, tail_ok, list(red.buckets), launched_before_finish, red.bucket))
    finally:
        dist.destroy_process_group()


def test_grad_reducer_unet_layout_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_unet_layout_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=180) for _ in range(world)], key=lambda r: r[0])
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    total = res[0][1]
    assert total == 7_834_588
    for rank, _, avg_ok, tail_ok, buckets, launched, bsz in res:
        assert tail_ok, rank
        assert avg_ok, rank                            # AVG of the two ranks' gradients
        # full buckets while the backward runs, in order, tiling [0, total) exactly; the tail at finish
        assert buckets[0][0] == 0 and buckets[-1][1] == total
        assert all(a[1] == b[0] for a, b in zip(buckets, buckets[1:]))
        assert all(hi - lo == bsz for lo, hi in buckets[:-1]) and 0 < buckets[-1][1] - buckets[-1][0] <= bsz
        assert launched == (total // bsz) * bsz
    assert res[0][4] == res[1][4]                      # identical bucket boundaries on both ranks


def _val_worker(rank, world, port, q, tmp):
    """train_model under DataParallel: every rank validates with rank 0's BN buffers, so the
    reduced val loss is the single-process loss of the model rank 0 checkpoints."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from superresolution_for_pdes_amd.distributed import DataParallel
        from superresolution_for_pdes_amd.train_enhanced import train_model

        class Tiny(torch.nn.Module):
            def __init__(self):
                super().__init__()
                self.lin = torch.nn.Linear(3, 4)
                self.bn = torch.nn.BatchNorm1d(4)

            def forward(self, x):
                return self.bn(self.lin(x))

        torch.manual_seed(0)
        t = Tiny()
        dp = DataParallel(t)
        g = torch.Generator().manual_seed(10 + rank)      # different training shards per rank
        train = [(torch.randn(8, 3, generator=g) * (rank + 1), torch.randn(8, 4, generator=g)) for _ in range(3)]
        gv = torch.Generator().manual_seed(99)            # the same validation set on every rank
        val_all = [(torch.randn(5, 3, generator=gv), torch.randn(5, 4, generator=gv)) for _ in range(4)]
        val = val_all[rank::world]                        # single-process batches dealt round-robin
        opt = torch.optim.SGD(t.parameters(), lr=0.0)     # parameters stay equal: only BN buffers differ
        sched = torch.optim.lr_scheduler.ReduceLROnPlateau(opt, mode="min", factor=0.5, patience=10)
        hist = train_model(dp, train, val, torch.nn.MSELoss(), opt, sched, 1, "cpu", tmp, None)
        t.eval()
        with torch.no_grad():
            want = sum(float(torch.nn.functional.mse_loss(t(x), y)) for x, y in val_all) / len(val_all)
        q.put((rank, hist["val_loss"][0], want, t.bn.running_mean.tolist()))
    finally:
        dist.destroy_process_group()


def test_val_loss_uses_rank0_buffers_world2(tmp_path):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_val_worker, args=(r, world, port, q, str(tmp_path))) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=180) for _ in range(world)], key=lambda r: r[0])
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, v0, want0, rm0), (_, v1, _, rm1) = res
    assert rm0 == rm1                                  # rank 1 validated with rank 0's buffers
    assert abs(v0 - want0) <= 1e-6 * max(1.0, abs(want0)), (v0, want0)
    assert v0 == v1


def _world1_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from superresolution_for_pdes_amd.distributed import DataParallel
        res = {}
        for keep in (False, True):
            m = torch.nn.Linear(3, 2)
            dp = DataParallel(m, reduce_single_rank=keep)
            red = m._grad_reducer
            calls = []
            orig = dist.all_reduce

            def spy(t, *a, **k):
                calls.append(t.numel())
                return orig(t, *a, **k)
            dist.all_reduce = spy
            try:
                flat = torch.arange(600, dtype=torch.float32)
                red.begin(flat)
                red.ready(600)
                red.finish()
            finally:
                dist.all_reduce = orig
            res[keep] = (calls, torch.equal(flat, torch.arange(600, dtype=torch.float32)), dp is not None)
        q.put(res)
    finally:
        dist.destroy_process_group()


def test_one_rank_group_keeps_collective_on_request():
    """Verdict r4 #7: a one-rank DataParallel skips the buckets' all-reduce by default; with
    reduce_single_rank=True (bench.py --ddp-rccl) every bucket still goes through the collective, and the
    gradient is unchanged (the mean over one rank)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_world1_worker, args=(0, 1, _free_port(), q))
    p.start()
    res = q.get(timeout=120)
    p.join(timeout=60)
    assert res[False][0] == [] and res[False][1]
    assert sum(res[True][0]) == 600 and len(res[True][0]) >= 1 and res[True][1]
