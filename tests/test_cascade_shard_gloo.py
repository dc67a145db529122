"""CPU, gloo world 2 and 3: the sharded cascade (SURVEY 8(e) row "Cascade (#5)") equals the
single-process cascade.  The U-Net is replaced by a per-tile stand-in and the HIP bilinear
by F.interpolate: this checks the subtree partition, block bookkeeping and the gather --
the kernels themselves are covered by tests/test_gpu_cascade.py."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn.functional as F


class _TileModel(torch.nn.Module):
    """Deterministic, position-independent per-tile map [T,3,40,40] -> [T,1,40,40]."""

    def forward(self, x):
        k = torch.tensor([[[[0.0, 0.1, 0.0], [0.1, 0.5, 0.1], [0.0, 0.1, 0.0]]]], dtype=x.dtype)
        return F.conv2d(x[:, 0:1], k, padding=1) + 0.01 * x[:, 2:3] * x[:, 1:2]


def _interp(x, ho, wo):
    return F.interpolate(x, size=(ho, wo), mode="bilinear", align_corners=True)


def _data(seed=0, start=20, target=160):
    rng = np.random.default_rng(seed)
    d = {"u": {}, "f": {}, "theta": {}}
    r = start
    while r <= target:
        d["u"][r] = rng.standard_normal((r, r)) * 1e-3
        d["f"][r] = rng.standard_normal((r, r))
        d["theta"][r] = rng.uniform(0.5, 2.0, (r, r))
        r *= 2
    return d


def _run(shard):
    from superresolution_for_pdes_amd import resolution_comparison as RC
    RC.upsample_bilinear = _interp
    return RC.ml_multi_level_upscale(_TileModel(), _data(), 160, device="cpu", start_resolution=20, shard=shard)


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
        q.put((rank, _run(None)))   # shard from the process group
    finally:
        dist.destroy_process_group()


def _spawn(world):
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
    return [r[1] for r in sorted(res, key=lambda t: t[0])]


def test_blocks_tiles_roundtrip():
    from superresolution_for_pdes_amd import resolution_comparison as RC
    b = torch.arange(2 * 80 * 80, dtype=torch.float64).reshape(2, 80, 80)
    t = RC._blocks_to_tiles(b, 20)
    assert t.shape == (32, 20, 20)
    assert torch.equal(t[5], b[0, 20:40, 20:40])       # block 0, tile (1, 1)
    assert torch.equal(t[16 + 3], b[1, 0:20, 60:80])   # block 1, tile (0, 3)
    assert torch.equal(RC._tiles_to_blocks(t, 2), b)
    assert torch.equal(RC._tiles_to_blocks(RC._blocks_to_tiles(b[:1], 20), 1), b[:1])


def test_sharded_cascade_equals_single_process():
    ref = _run((0, 1))
    assert ref.shape == (160, 160)
    # CPU conv2d picks batch-size dependent blockings, so per-tile results differ in the last
    # fp32 bits between batch compositions; a misplaced block would be an O(1) error
    tol = 1e-5 * float(np.abs(ref).max())
    for world in (2, 3):          # 16 level-2 roots: 8+8, and the uneven 6+5+5
        for out in _spawn(world):
            np.testing.assert_allclose(out, ref, rtol=0, atol=tol)
