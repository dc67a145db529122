"""Scheduling variants of the HIP path give bit-identical results.

Every kernel on the path is deterministic (fixed-order reductions, no float atomics), so
moving launches between streams (unet_exec.WgradStream: weight gradients on a side stream)
or changing which kernel computes a tile (the register-staged h3r kernel against the 8-wave one,
SRPDE_FAM_NO_H3R) must not change a single bit.  Anything else is a race or a
wrong tile, which a tolerance-based parity test could hide.
"""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _train_step(x, state, wgrad_stream, priority=False):
    from superresolution_for_pdes_amd import unet_exec
    from superresolution_for_pdes_amd.models import UNet
    saved = unet_exec._WGRAD_STREAM, unet_exec._BWD_PRIORITY
    unet_exec._WGRAD_STREAM, unet_exec._BWD_PRIORITY = wgrad_stream, ("1" if priority else "0")
    try:
        m = UNet()
        m.load_state_dict(state)
        m = m.to(DEV).train()
        out = m(x)
        (out ** 2).mean().backward()
        torch.cuda.synchronize()
        grads = {n: p.grad.detach().clone() for n, p in m.named_parameters()}
        bufs = {n: b.detach().clone() for n, b in m.named_buffers()}
    finally:
        unet_exec._WGRAD_STREAM, unet_exec._BWD_PRIORITY = saved
    return out.detach(), grads, bufs


def test_wgrad_side_stream_is_bit_identical():
    from superresolution_for_pdes_amd.models import UNet, init_weights
    torch.manual_seed(0)
    ref = UNet()
    ref.apply(init_weights)
    state = {k: v.clone() for k, v in ref.state_dict().items()}
    x = torch.randn(16, 3, 40, 40, generator=torch.Generator().manual_seed(5)).to(DEV)
    x[:, 1] = 1.0
    a = _train_step(x, state, False)
    for b in (_train_step(x, state, True), _train_step(x, state, True, priority=True)):
        assert torch.equal(a[0], b[0])
        for n in a[1]:
            assert torch.equal(a[1][n], b[1][n]), n
        for n in a[2]:
            assert torch.equal(a[2][n], b[2][n]), n


def test_data_parallel_world1_is_bit_identical():
    """DataParallel over a one-rank RCCL group (bucketed all-reduce on the reducer stream, the
    dgrad chain on the high-priority stream it selects by default) == the plain step, bit for bit
    (AVG over one rank multiplies by 1)."""
    import os
    import socket
    import torch.distributed as dist
    from superresolution_for_pdes_amd.distributed import DataParallel
    from superresolution_for_pdes_amd.models import UNet, init_weights
    torch.manual_seed(1)
    ref = UNet()
    ref.apply(init_weights)
    state = {k: v.clone() for k, v in ref.state_dict().items()}
    x = torch.randn(16, 3, 40, 40, generator=torch.Generator().manual_seed(6)).to(DEV)
    x[:, 1] = 1.0
    a = _train_step(x, state, True)
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device(DEV, torch.cuda.current_device()))
    try:
        m = UNet()
        m.load_state_dict(state)
        m = m.to(DEV).train()
        net = DataParallel(m, bucket_bytes=1 << 20)   # several buckets during the backward
        out = net(x)
        (out ** 2).mean().backward()
        torch.cuda.synchronize()
        assert torch.equal(a[0], out.detach())
        for n, p in m.named_parameters():
            assert torch.equal(a[1][n], p.grad), n
    finally:
        dist.destroy_process_group()


def test_reducer_buckets_wait_for_their_gradients():
    """World-1 stand-in for the data-parallel reducer whose "collective" scales its bucket by 3 on
    the reducer stream.  A bucket launched before every kernel writing into it finished (dgrad-chain
    BN / head gradients on the high-priority stream, wgrad and attention parameter gradients on the
    side stream) would be overwritten unscaled: the gradients must equal exactly 3x the plain ones."""
    from superresolution_for_pdes_amd.distributed import GradReducer
    from superresolution_for_pdes_amd.models import UNet, init_weights

    class ScaleReducer(GradReducer):
        def __init__(self, bucket_bytes):   # no process group
            self.pg, self.bucket, self.world, self.backend, self.use_avg = None, bucket_bytes // 4, 1, "fake", True
            self.flat, self.launched, self.works, self.stream = None, 0, [], None
            self.n_buckets, self.buckets, self.wait_streams = 0, [], ()

        def _collective(self, chunk):
            chunk.mul_(3.0)
            return None

    torch.manual_seed(2)
    ref = UNet()
    ref.apply(init_weights)
    state = {k: v.clone() for k, v in ref.state_dict().items()}
    x = torch.randn(16, 3, 40, 40, generator=torch.Generator().manual_seed(7)).to(DEV)
    x[:, 1] = 1.0
    a = _train_step(x, state, True)
    m = UNet()
    m.load_state_dict(state)
    m = m.to(DEV).train()
    m._grad_reducer = ScaleReducer(1 << 20)
    out = m(x)
    (out ** 2).mean().backward()
    torch.cuda.synchronize()
    assert m._grad_reducer.n_buckets >= 8
    assert torch.equal(a[0], out.detach())
    for n, p in m.named_parameters():
        assert torch.equal(a[1][n] * 3.0, p.grad), n


@pytest.mark.parametrize("n,c0,c1,cout,hw,dil", [(4, 64, 0, 64, 40, 1), (5, 128, 64, 64, 40, 1), (3, 64, 0, 32, 40, 1),
                                                 (4, 32, 0, 16, 40, 1), (6, 128, 0, 64, 20, 1), (2, 64, 0, 64, 10, 2)])
def test_conv_h3r_equals_8wave(n, c0, c1, cout, hw, dil):
    """The register-staged 4-wave h3 kernel (two workgroups per CU) against the 8-wave kernel:
    forward (bias, BN statistics, stored input split, fused input BN + ReLU) and dgrad (stored
    dy split, fused BN-backward partials, per-tile max|dx|) in equal bits -- same products, same
    accumulation order, statistics combined per 32-row block in row order (no K-split tail at
    these sizes)."""
    from superresolution_for_pdes_amd import hipops as H
    cin = c0 + c1
    if H.conv_math() != "h3" or not H.h3_capable(c0, c1, cout, hw, dil):
        pytest.skip("not an h3 shape")
    back = H.h3_capable(cout, 0, cin, hw, dil)   # out_conv2's 16-channel dy: forward only
    g = torch.Generator(device=DEV).manual_seed(5)
    P = n * hw * hw
    x = torch.randn(P, cin, device=DEV, generator=g)
    x0, x1 = (x[:, :c0], x[:, c0:]) if c1 else (x, None)
    w = torch.randn(cout, cin, 3, 3, device=DEV, generator=g) * 0.05
    b = torch.randn(cout, device=DEV, generator=g)
    wf, wd = H.pack_conv_weights(w, cin, True, back)
    dy = torch.randn(P, cout, device=DEV, generator=g)
    by = torch.randn(P, cin, device=DEV, generator=g)        # the BN input below the dgrad's output
    bmean, binv = torch.randn(cin, device=DEV, generator=g) * 0.1, torch.rand(cin, device=DEV, generator=g) + 0.5
    bga, bbe = torch.randn(cin, device=DEV, generator=g), torch.randn(cin, device=DEV, generator=g) * 0.1
    for t in (x0, x1, dy):
        if t is not None:
            t._srpde_amax = H.amax_of(t)
    aff = None
    if c1 == 0:   # fused input BN + ReLU (the second conv of a ConvBlock)
        sc = torch.rand(c0, device=DEV, generator=g) + 0.5
        sh = torch.randn(c0, device=DEV, generator=g) * 0.2
        aff = (sc, sh)
    outs = []
    prev = H.set_h3r(True)
    try:
        for on in (False, True):
            H.set_h3r(on)
            y = torch.empty(P, cout, device=DEV)
            stats, _, _ = H.conv_stats_buffer(n, hw, hw, cout, DEV, c0, c1, dil)
            xp = H.split_planes_buffer(P, cin, DEV)
            H.conv_fwd(x0, x1, wf, b, y, n, hw, hw, cout, 3, dil, 1, False, stats, xp, in_affine=aff)
            dx = dyp = part = dmax = torch.zeros(1, device=DEV)
            if back:
                dx = torch.empty(P, cin, device=DEV)
                dyp = H.split_planes_buffer(P, cout, DEV)
                part = H.bn_bwd_partials(n, hw, hw, cin, DEV)
                dmax = H.out_max_slots(n, hw, hw, cout, cin, dil, DEV)
                H.conv_fwd(dy, None, wd, None, dx, n, hw, hw, cin, 3, dil, -1, False, None, dyp,
                           bn_bwd=(by, bmean, binv, bga, bbe, part), out_max=dmax)
            torch.cuda.synchronize()
            outs.append((y, stats, xp, dx, dyp, part, dmax))
    finally:
        H.set_h3r(prev)
    names = ("y", "stats", "xsplit", "dx", "dysplit", "bn_part", "dx_max")
    for name, a, b_ in zip(names, *outs):
        assert torch.equal(a, b_), name
