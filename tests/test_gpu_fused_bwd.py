"""Fused backward reductions.  The encoder outputs' gradient in one pass (srpde_att_pool_bn_bwd): e1 / e2 = relu(bn2(y)) of enc1 / enc2 feed the
AttentionGate of their skip connection and the next block's 2x2 max-pool (src/models.py:79-80, 90, 93, 119-130), so
their gradient is the gate's input gradient plus the max-pool backward, and enc*.bn2's backward reduces over it.
The fused kernel writes that gradient once and emits the reduction's partial sums; the executor's three-pass path
(att_bwd dx, maxpool_bwd accumulate, bn_bwd_prepare's own reduction) is the reference: e2's gradient must be EQUAL
bit for bit (same expressions, same order), e1's and every parameter gradient within fp32 summation-order rounding."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _step(model, x, t, fuse, attr="_FUSE_ENC_OUT", keep=("e1", "e2")):
    from superresolution_for_pdes_amd import unet_exec as X
    from superresolution_for_pdes_amd.functional import mse_loss
    prev = getattr(X, attr)
    setattr(X, attr, fuse)
    X.DEBUG_TAPS = {}
    try:
        for p in model.parameters():
            p.grad = None
        loss = mse_loss(model(x), t)
        loss.backward()
        torch.cuda.synchronize()
        taps = X.DEBUG_TAPS
    finally:
        X.DEBUG_TAPS = None
        setattr(X, attr, prev)
    return {k: v for k, v in taps.items() if k in keep}, {n: p.grad.clone() for n, p in model.named_parameters()}


@pytest.mark.parametrize("n", [4, 37])
def test_fused_encoder_output_backward_matches_three_passes(n):
    from oracle import unet_ref as U   # (test infrastructure: the seeded reference initialisation)
    from superresolution_for_pdes_amd.models import UNet
    st = U.kaiming_init_state(3)
    model = UNet()
    model.load_state_dict(st)
    model = model.to(DEV).train()
    g = torch.Generator(device=DEV).manual_seed(11 + n)
    x = torch.randn(n, 3, 40, 40, device=DEV, generator=g)
    x[:, 1] = 1.0
    t = torch.randn(n, 1, 40, 40, device=DEV, generator=g)
    taps_f, grads_f = _step(model, x, t, True)
    taps_u, grads_u = _step(model, x, t, False)
    # e2's inputs are the same on both paths: equal bit for bit.  e1 reads dp1, enc2's input gradient, which
    # follows enc2.bn2's reduction (summed in another order on the fused path): fp32 rounding apart
    assert torch.equal(taps_f["e2"], taps_u["e2"])
    d1 = float((taps_f["e1"] - taps_u["e1"]).double().norm() / taps_u["e1"].double().norm())
    assert d1 < 1e-5, d1
    worst = 0.0
    for name, gu in grads_u.items():
        gf = grads_f[name]
        if name.endswith("conv1.bias") or name.endswith("conv2.bias"):
            continue   # BN-fed conv biases: true gradient 0, rounding noise only
        rel = float((gf - gu).double().norm() / max(float(gu.double().norm()), 1e-30))
        worst = max(worst, rel)
        assert rel < 2e-5, (name, rel)
    print(f"worst parameter-gradient relative difference {worst:.2e}")


@pytest.mark.parametrize("n", [3, 33])
def test_upsample_backward_bn_reduction_matches_separate_pass(n):
    """dec2.bn2 / dec3.bn2's backward reduction formed by the upsample backward that writes their output
    gradient (srpde_upsample_bilinear_bwd_gated_bn) against the separate reduction pass: the upsample's output
    (d2) EQUAL bit for bit, d3 (after dec2's backward) and every parameter gradient within fp32 summation-order rounding."""
    from oracle import unet_ref as U   # (test infrastructure: the seeded reference initialisation)
    from superresolution_for_pdes_amd.models import UNet
    model = UNet()
    model.load_state_dict(U.kaiming_init_state(5))
    model = model.to(DEV).train()
    g = torch.Generator(device=DEV).manual_seed(7 + n)
    x = torch.randn(n, 3, 40, 40, device=DEV, generator=g)
    x[:, 1] = 1.0
    t = torch.randn(n, 1, 40, 40, device=DEV, generator=g)
    taps_f, grads_f = _step(model, x, t, True, "_FUSE_UP_BN", ("d2", "d3"))
    taps_u, grads_u = _step(model, x, t, False, "_FUSE_UP_BN", ("d2", "d3"))
    assert set(taps_f) == {"d2", "d3"}
    assert torch.equal(taps_f["d2"], taps_u["d2"])   # written before any changed reduction is read
    d3 = float((taps_f["d3"] - taps_u["d3"]).double().norm() / taps_u["d3"].double().norm())
    assert d3 < 1e-5, d3
    worst = 0.0
    for name, gu in grads_u.items():
        if name.endswith(("conv1.bias", "conv2.bias")) or name in ("bridge.0.bias", "bridge.3.bias"):
            continue   # BN-fed conv biases: true gradient 0, rounding noise only
        rel = float((grads_f[name] - gu).double().norm() / max(float(gu.double().norm()), 1e-30))
        worst = max(worst, rel)
        assert rel < 2e-5, (name, rel)
    print(f"worst parameter-gradient relative difference {worst:.2e}")


def test_upsample_bn_partials_match_bn_reduction():
    """The kernel's partials and max|dx| slots, summed, equal bn_bwd_prepare's own reduction pass on the same
    (y, dx) to fp32 rounding: dgamma / dbeta and the m1 / m2 terms."""
    from superresolution_for_pdes_amd import hipops as H
    n, h, w, c = 6, 20, 20, 128
    ho, wo = 2 * h, 2 * w
    g = torch.Generator(device=DEV).manual_seed(3)
    dout = torch.randn(n * ho * wo, c, device=DEV, generator=g)
    dsa = torch.randn(n * ho * wo, device=DEV, generator=g)
    wg = torch.randn(c, device=DEV, generator=g)
    y = torch.randn(n * h * w, c, device=DEV, generator=g)
    mean = y.mean(0)
    invstd = 1.0 / (y.var(0, unbiased=False) + 1e-5).sqrt()
    gamma = torch.rand(c, device=DEV, generator=g) + 0.5
    beta = torch.randn(c, device=DEV, generator=g) * 0.1
    dx_a, dx_b = H.empty(n * h * w, c, device=DEV), H.empty(n * h * w, c, device=DEV)
    part, da_max = H.upsample_bwd(dout, dx_a, n, h, w, ho, wo, False, gate=(dsa, wg), bn=(y, mean, invstd, gamma, beta))
    assert H.upsample_bwd(dout, dx_b, n, h, w, ho, wo, False, gate=(dsa, wg)) is None
    torch.cuda.synchronize()
    assert torch.equal(dx_a, dx_b)
    assert float(da_max.max()) == float(dx_a.abs().max())
    outs = []
    for pt in ((part, da_max), None):
        dg, db, dbias = (torch.empty(c, device=DEV) for _ in range(3))
        m1, m2, word = H.bn_bwd_prepare(y, dx_a, mean, invstd, gamma, beta, dg, db, dbias,
                                        part=None if pt is None else pt[0], da_max=None if pt is None else pt[1])
        outs.append((dg, db, m1, m2))
    for a, b in zip(*outs):
        rel = float((a - b).double().norm() / b.double().norm())
        assert rel < 1e-5, rel


@pytest.mark.parametrize("n", [2, 17])
def test_gating_bn_reduction_matches_separate_passes(n):
    """bridge[4]'s backward reduction formed with att3's gating gradient (srpde_gating_bn_reduce) against the
    att_bwd dg pass plus a separate reduction: db (the bridge output's gradient) within fp32 rounding of the
    same sum, every parameter gradient within summation-order rounding."""
    from oracle import unet_ref as U   # (test infrastructure: the seeded reference initialisation)
    from superresolution_for_pdes_amd.models import UNet
    model = UNet()
    model.load_state_dict(U.kaiming_init_state(9))
    model = model.to(DEV).train()
    g = torch.Generator(device=DEV).manual_seed(21 + n)
    x = torch.randn(n, 3, 40, 40, device=DEV, generator=g)
    x[:, 1] = 1.0
    t = torch.randn(n, 1, 40, 40, device=DEV, generator=g)
    taps_f, grads_f = _step(model, x, t, True, "_FUSE_GATING_BN", ("b",))
    taps_u, grads_u = _step(model, x, t, False, "_FUSE_GATING_BN", ("b",))
    db = float((taps_f["b"] - taps_u["b"]).double().norm() / taps_u["b"].double().norm())
    assert db < 1e-6, db
    worst = 0.0
    for name, gu in grads_u.items():
        if name.endswith(("conv1.bias", "conv2.bias")) or name in ("bridge.0.bias", "bridge.3.bias"):
            continue   # BN-fed conv biases: true gradient 0, rounding noise only
        rel = float((grads_f[name] - gu).double().norm() / max(float(gu.double().norm()), 1e-30))
        worst = max(worst, rel)
        assert rel < 2e-5, (name, rel)
    print(f"db {db:.2e}, worst parameter-gradient relative difference {worst:.2e}")


def test_gating_bn_partials_match_bn_reduction():
    """srpde_gating_bn_reduce's dg equals dg + dsa (x) wg formed in fp64 to fp32 rounding, and its partials /
    max slots give bn_bwd_prepare the terms of its own reduction pass."""
    from superresolution_for_pdes_amd import hipops as H
    P, C = 4 * 100, 512
    g = torch.Generator(device=DEV).manual_seed(4)
    dsa = torch.randn(P, device=DEV, generator=g)
    wg = torch.randn(C, device=DEV, generator=g)
    dg0 = torch.randn(P, C, device=DEV, generator=g)
    y = torch.randn(P, C, device=DEV, generator=g)
    mean = y.mean(0)
    invstd = 1.0 / (y.var(0, unbiased=False) + 1e-5).sqrt()
    gamma = torch.rand(C, device=DEV, generator=g) + 0.5
    beta = torch.randn(C, device=DEV, generator=g) * 0.1
    dg = dg0.clone()
    part, da_max = H.gating_bn_reduce(dsa, wg, dg, y, mean, invstd, gamma, beta)
    torch.cuda.synchronize()
    ref = dg0.double() + dsa.double()[:, None] * wg.double()[None, :]
    assert float((dg.double() - ref).abs().max()) <= 4e-7 * float(ref.abs().max())
    assert float(da_max.max()) == float(dg.abs().max())
    outs = []
    for pt in ((part, da_max), None):
        dgm, db, dbias = (torch.empty(C, device=DEV) for _ in range(3))
        m1, m2, word = H.bn_bwd_prepare(y, dg, mean, invstd, gamma, beta, dgm, db, dbias,
                                        part=None if pt is None else pt[0], da_max=None if pt is None else pt[1])
        outs.append((dgm, db, m1, m2))
    for a, b in zip(*outs):
        rel = float((a - b).double().norm() / b.double().norm())
        assert rel < 1e-5, rel


@pytest.mark.parametrize("n", [3, 21])
def test_gate_weight_gradient_from_low_res(n):
    """The decoder gates' spatial-conv weight / bias gradients formed from the low-res decoder output
    (srpde_att_bwd_params_lowres: sum_q d[q] up^T(dsa)[q]) against the sum over the upsampled g = up(d): the same
    sum regrouped -- every parameter gradient within fp32 summation-order rounding."""
    from oracle import unet_ref as U   # (test infrastructure: the seeded reference initialisation)
    from superresolution_for_pdes_amd.models import UNet
    model = UNet()
    model.load_state_dict(U.kaiming_init_state(17))
    model = model.to(DEV).train()
    g = torch.Generator(device=DEV).manual_seed(41 + n)
    x = torch.randn(n, 3, 40, 40, device=DEV, generator=g)
    x[:, 1] = 1.0
    t = torch.randn(n, 1, 40, 40, device=DEV, generator=g)
    _, grads_f = _step(model, x, t, True, "_GATE_WGRAD_LOWRES", ())
    _, grads_u = _step(model, x, t, False, "_GATE_WGRAD_LOWRES", ())
    worst = {}
    for name, gu in grads_u.items():
        if name.endswith(("conv1.bias", "conv2.bias")) or name in ("bridge.0.bias", "bridge.3.bias"):
            continue   # BN-fed conv biases: true gradient 0, rounding noise only
        rel = float((grads_f[name] - gu).double().norm() / max(float(gu.double().norm()), 1e-30))
        worst[name] = rel
        assert rel < 2e-5, (name, rel)
    gate = {k: v for k, v in worst.items() if "spatial_attention" in k}
    assert len(gate) >= 4 and any(v > 0 for v in gate.values())   # the path really changed those sums
    print({k: f"{v:.1e}" for k, v in gate.items()})


@pytest.mark.parametrize("n", [2, 19])
def test_enc1_conv1_weight_gradient_with_fused_bn_backward(n):
    """enc1.conv1's fp32 weight gradient applying enc1.bn1's backward to its dY loads (srpde_conv_wgrad_bnb)
    against dy written by bn_relu_bwd and read back: the same dy bits, so the weight gradient is EQUAL bit for bit,
    and so is every other gradient but the BN-fed conv bias (formed analytically instead of summed)."""
    from oracle import unet_ref as U   # (test infrastructure: the seeded reference initialisation)
    from superresolution_for_pdes_amd.models import UNet
    model = UNet()
    model.load_state_dict(U.kaiming_init_state(23))
    model = model.to(DEV).train()
    g = torch.Generator(device=DEV).manual_seed(51 + n)
    x = torch.randn(n, 3, 40, 40, device=DEV, generator=g)
    x[:, 1] = 1.0
    t = torch.randn(n, 1, 40, 40, device=DEV, generator=g)
    _, grads_f = _step(model, x, t, True, "_FUSE_WGRAD_BN", ())
    _, grads_u = _step(model, x, t, False, "_FUSE_WGRAD_BN", ())
    for name, gu in grads_u.items():
        if name == "enc1.conv1.bias":
            rel = float((grads_f[name] - gu).double().norm() / max(float(grads_u["enc1.conv1.weight"].norm()), 1e-30))
            assert rel < 1e-5, rel   # true gradient 0: rounding noise either way
            continue
        assert torch.equal(grads_f[name], gu), name
