"""srpde_conv_wgrad_h3x: the 40 x 40 layers' weight gradient splitting its fp32 input rows itself (fused input
BN + ReLU of x0, attention gate of x1, the forward's scale) instead of reading the split the training
forward stored (src/models.py:16,18,57,59 -- enc1.conv2, dec1.conv1, dec1.conv2, out_conv1, out_conv2 --
through aten::convolution_backward's weight gradient).  The staged operand is the forward's split bit for
bit, so dw must EQUAL srpde_conv_wgrad_h3p's on the stored split; it is also held to fp64.  End to end: the
train step with the stored splits (unet_exec._WGRAD_X off) and without gives the same gradients bit for bit."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rows(x):
    n, c, h, w = x.shape
    return x.permute(0, 2, 3, 1).reshape(n * h * w, c).contiguous()


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


@pytest.mark.parametrize("n,h,c0,c1,cout,dil,mode", [
    (3, 40, 64, 0, 64, 1, "aff"),      # enc1.conv2 / dec1.conv2: fused input BN + ReLU
    (2, 40, 128, 64, 64, 1, "gate"),   # dec1.conv1: [up(d2), att1(e1)], gated second input
    (3, 40, 64, 0, 32, 1, "aff"),      # out_conv1
    (3, 40, 32, 0, 16, 1, "aff"),      # out_conv2 (16 outputs: 32-channel dy planes)
    (1, 40, 64, 0, 64, 1, "plain"),    # one sample: a single split, ragged tail
    (5, 13, 64, 0, 64, 1, "plain"),    # not the h5 width: the h3 forward's split
    (2, 20, 64, 32, 32, 2, "plain"),   # dilation 2, plain concat
    (7, 40, 64, 0, 64, 1, "gate0"),    # x0 only, a gate object absent
])
def test_wgrad_h3x_equals_stored_split(n, h, c0, c1, cout, dil, mode, conv_math):
    from superresolution_for_pdes_amd import hipops as H
    H.set_conv_math("h3")
    cin = c0 + c1
    w_ = h
    assert H.wgrad_x_capable(c0, c1, cout, w_, dil)
    g = torch.Generator().manual_seed(n * 7 + cin + cout)
    x = torch.randn(n, cin, h, w_, generator=g, dtype=torch.float64)
    wt = torch.randn(cout, cin, 3, 3, generator=g, dtype=torch.float64) * (2.0 / (9 * cin)) ** 0.5
    dy = torch.randn(n, cout, h, w_, generator=g, dtype=torch.float64) * 1e-3
    P = n * h * w_
    aff = gate = None
    xe = x.clone()   # the conv's effective input
    if mode == "aff":
        s = torch.rand(c0, generator=g, dtype=torch.float64) + 0.5
        t = torch.randn(c0, generator=g, dtype=torch.float64) * 0.3
        aff = (s.float().to(DEV), t.float().to(DEV))
        xe = torch.relu(x.float() * s.float().view(1, -1, 1, 1) + t.float().view(1, -1, 1, 1)).double()
    elif mode == "gate":
        ca = torch.sigmoid(torch.randn(n, c1, generator=g)).double()
        sa = torch.sigmoid(torch.randn(n, 1, h, w_, generator=g)).double()
        gate = (ca.float().to(DEV).contiguous(), _rows(sa.float()).view(-1).to(DEV).contiguous())
        xe[:, c0:] = ((x[:, c0:].float() * ca.float().view(n, c1, 1, 1)) * sa.float()).double()
    xr = _rows(x.float()).to(DEV)
    x0, x1 = (xr[:, :c0], xr[:, c0:]) if c1 else (xr, None)
    if mode == "aff":   # the producer's max|relu(bn(y))| word, as the training forward tags it
        x0 = x0.clone()
        x0._srpde_amax = torch.tensor([float(xe.abs().max())], dtype=torch.float32).view(torch.int32).to(DEV)
    wf, wd = H.pack_conv_weights(wt.float().to(DEV), cin, want_dgrad=True)
    cp = H.cpad32(cout)
    xp, dyp = H.split_planes_buffer(P, cin, DEV), H.split_planes_buffer(P, cp, DEV)
    y = H.empty(P, cout, device=DEV)
    H.conv_fwd(x0, x1, wf, None, y, n, h, w_, cout, 3, dil, 1, False, None, xp, in_affine=aff, x1_gate=gate)
    dyr = _rows(dy.float()).to(DEV)
    dyin = dyr if cp == cout else torch.cat([dyr, torch.zeros(P, cp - cout, device=DEV)], 1)
    dx = H.empty(P, cin, device=DEV)
    H.conv_fwd(dyin, None, wd, None, dx, n, h, w_, cin, 3, dil, -1, False, None, dyp)
    dw_p = torch.empty(cout, cin, 3, 3, device=DEV)
    H.conv_wgrad_h3p(dyp, xp, dw_p, n, h, w_, 3, dil)
    dw_x = torch.full((cout, cin, 3, 3), float("nan"), device=DEV)
    H.conv_wgrad_h3p(dyp, H.XSource(x0, x1, aff, gate), dw_x, n, h, w_, 3, dil)
    assert H.query("srpde_last_kernel").decode().startswith("conv_wgrad_h3h_kernel<")
    torch.cuda.synchronize()
    assert torch.equal(dw_x, dw_p), float((dw_x - dw_p).abs().max())
    dw64 = torch.nn.grad.conv2d_weight(xe, wt.shape, dy, padding=dil, dilation=dil)
    assert _rel(dw_x, dw64) < 1e-6


def test_wgrad_h3x_rejects_unsupported_shapes():
    from superresolution_for_pdes_amd import hipops as H
    assert not H.wgrad_x_capable(128, 0, 128, 20, 1)    # Cout > 64: h3p's tiles
    assert not H.wgrad_x_capable(48, 0, 64, 40, 1)      # a 32-channel chunk would straddle the inputs
    assert not H.wgrad_x_capable(64, 0, 64, 200, 1)     # the row ring cannot hold a stage's reach
    assert H.wgrad_x_capable(128, 64, 64, 40, 1) and H.wgrad_x_capable(32, 0, 16, 40, 1)


def test_train_step_without_stored_splits_is_bit_identical():
    """unet_exec._WGRAD_X: the 40 x 40 training forwards store no input split and their weight gradients
    split the input rows themselves -- every gradient, the input gradient and the output equal the
    stored-split path's bit for bit (B = 6: several splits per layer)."""
    import sys
    import os
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from branch import hip_step
    from state import fixture_state_torch
    from superresolution_for_pdes_amd import unet_exec
    from superresolution_for_pdes_amd.models import UNet
    g = torch.Generator().manual_seed(11)
    x = torch.randn(6, 3, 40, 40, generator=g)
    x[:, 1] = 1.0
    t = torch.randn(6, 1, 40, 40, generator=g)
    saved = unet_exec._WGRAD_X
    res = []
    try:
        for on in (False, True):
            unet_exec._WGRAD_X = on
            m = UNet()
            m.load_state_dict(fixture_state_torch())
            m = m.to(DEV).train(True)
            m.flatten_parameters_()
            out, grads, dx, _ = hip_step(m, x.to(DEV), t.to(DEV))
            res.append((out.detach().clone(), {k: v.detach().clone() for k, v in grads.items()}, dx.clone()))
    finally:
        unet_exec._WGRAD_X = saved
    (o0, g0, d0), (o1, g1, d1) = res
    assert torch.equal(o0, o1) and torch.equal(d0, d1)
    diff = [k for k in g0 if not torch.equal(g0[k], g1[k])]
    assert not diff, diff
