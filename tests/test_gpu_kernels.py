"""Per-kernel parity: libsrpde_hip.so vs plain PyTorch fp32 (CPU) of the same op.

Tolerances are relative to the op's magnitude; the fp32 MFMA conv sums in a different
order than mkldnn, so agreement is ~1e-6 relative, not bitwise.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rows(x):  # NCHW -> [P, C] NHWC rows
    n, c, h, w = x.shape
    return x.permute(0, 2, 3, 1).reshape(n * h * w, c).contiguous()


def unrows(r, n, h, w):
    return r.reshape(n, h, w, -1).permute(0, 3, 1, 2)


def rel(a, b):
    a = a.double().cpu()
    b = b.double().cpu()
    return float((a - b).norm() / max(b.norm(), 1e-30))


@pytest.mark.parametrize("n,cin0,cin1,cout,h,dil", [
    (2, 64, 0, 64, 40, 1), (3, 128, 0, 256, 10, 1), (2, 256, 0, 512, 10, 2), (2, 512, 256, 256, 10, 1),
    (2, 128, 64, 64, 40, 1), (2, 32, 0, 16, 40, 1), (2, 64, 0, 32, 40, 1), (1, 4, 0, 64, 40, 1),
    (3, 256, 128, 128, 20, 1), (5, 16, 0, 128, 6, 1),
    # ragged: P % 32 != 0, Cout not a tile multiple, K = 864 not a tile multiple, dil 2 on 7x7
    (3, 64, 32, 96, 7, 2), (16, 128, 0, 128, 20, 1)])
@pytest.mark.parametrize("math", ["h3", "f32"])
def test_conv_fwd_dgrad_wgrad(n, cin0, cin1, cout, h, dil, math, conv_math):
    from superresolution_for_pdes_amd import hipops as H
    H.set_conv_math(math)
    g = torch.Generator().manual_seed(n * 1000 + cout + cin0)
    cin = cin0 + cin1
    x = torch.randn(n, cin, h, h, generator=g)
    wt = torch.randn(cout, cin, 3, 3, generator=g) * (2.0 / (9 * cin)) ** 0.5
    b = torch.randn(cout, generator=g) * 0.1
    y_ref = F.conv2d(x, wt, b, padding=dil, dilation=dil)
    xr = rows(x).to(DEV)
    x0, x1 = (xr[:, :cin0], xr[:, cin0:]) if cin1 else (xr, None)
    wd = wt.to(DEV)
    wf, wdg = H.pack_conv_weights(wd, cin, want_dgrad=True)
    y = H.empty(n * h * h, cout, device=DEV)
    stats, nblk, rpb = H.conv_stats_buffer(n, h, h, cout, DEV, cin0, cin1, dil)
    H.conv_fwd(x0, x1, wf, b.to(DEV), y, n, h, h, cout, 3, dil, 1, False, stats)
    torch.cuda.synchronize()
    assert rel(unrows(y, n, h, h), y_ref) < 2e-6
    # BN statistics from the epilogue partials
    mean, invstd = H.bn_train_finalize(stats, nblk, rpb, n * h * h, None, None, None, 0.1, 1e-5)
    yr = y_ref.double()
    m_ref = yr.mean(dim=(0, 2, 3))
    v_ref = yr.var(dim=(0, 2, 3), unbiased=False)
    assert rel(mean, m_ref) < 1e-5
    assert rel(invstd, 1.0 / torch.sqrt(v_ref + 1e-5)) < 1e-5
    # dgrad + wgrad against autograd
    dy = torch.randn(n, cout, h, h, generator=g)
    xg = x.clone().requires_grad_(True)
    wg = wt.clone().requires_grad_(True)
    F.conv2d(xg, wg, None, padding=dil, dilation=dil).backward(dy)
    dyr = rows(dy).to(DEV)
    dx = H.empty(n * h * h, cin, device=DEV)
    H.conv_fwd(dyr, None, wdg, None, dx, n, h, h, cin, 3, dil, -1, False, None)
    dw = torch.empty_like(wd)
    H.conv_wgrad(dyr, x0, x1, dw, n, h, h, 3, dil)
    torch.cuda.synchronize()
    assert rel(unrows(dx, n, h, h), xg.grad) < 2e-6
    assert rel(dw, wg.grad) < 2e-6


@pytest.mark.parametrize("cin0,cin1,cout,h,dil", [(512, 0, 512, 10, 2), (128, 64, 64, 40, 1), (64, 0, 32, 40, 1)])
def test_conv_split_kernels_are_fp32_accurate(cin0, cin1, cout, h, dil, conv_math):
    """The split-operand conv against fp64: the scaled fp16 two-piece (h3) kernels must sit at the
    fp32 kernel's error level (far below the 2^-16-relative error of a 2-piece bf16 split).  Bars:
    < 1e-6 relative L2, and within 3x of the fp32-MFMA kernel's own error (+1e-7)."""
    from superresolution_for_pdes_amd import hipops as H
    g = torch.Generator().manual_seed(cin0 + cout)
    n, cin = 4, cin0 + cin1
    x = torch.randn(n, cin, h, h, generator=g, dtype=torch.float64)
    wt = torch.randn(cout, cin, 3, 3, generator=g, dtype=torch.float64) * (2.0 / (9 * cin)) ** 0.5
    y64 = F.conv2d(x, wt, None, padding=dil, dilation=dil)
    dy = torch.randn(n, cout, h, h, generator=g, dtype=torch.float64)
    dx64 = torch.nn.grad.conv2d_input(x.shape, wt, dy, padding=dil, dilation=dil)
    dw64 = torch.nn.grad.conv2d_weight(x, wt.shape, dy, padding=dil, dilation=dil)
    xr = rows(x.float()).to(DEV)
    x0, x1 = (xr[:, :cin0], xr[:, cin0:]) if cin1 else (xr, None)
    dyr = rows(dy.float()).to(DEV)
    errs = {}
    for math in ("f32", "h3"):
        H.set_conv_math(math)
        wf, wd = H.pack_conv_weights(wt.float().to(DEV), cin, want_dgrad=True)
        y = H.empty(n * h * h, cout, device=DEV)
        H.conv_fwd(x0, x1, wf, None, y, n, h, h, cout, 3, dil, 1, False, None)
        dx = H.empty(n * h * h, cin, device=DEV)
        H.conv_fwd(dyr, None, wd, None, dx, n, h, h, cin, 3, dil, -1, False, None)
        dw = torch.empty(cout, cin, 3, 3, device=DEV)
        H.conv_wgrad(dyr, x0, x1, dw, n, h, h, 3, dil)
        torch.cuda.synchronize()
        errs[math] = (rel(unrows(y, n, h, h), y64), rel(unrows(dx, n, h, h), dx64), rel(dw, dw64))
    print(f"conv fp64 errors (fwd, dgrad, wgrad): {errs}")
    for k in range(3):
        assert errs["h3"][k] < 1e-6, errs
        assert errs["h3"][k] < 3.0 * errs["f32"][k] + 1e-7, errs


def test_conv_cin_pad_and_accumulate():
    """enc1.conv1: 3 real input channels padded to 4; accumulate flag adds into the output."""
    from superresolution_for_pdes_amd import hipops as H
    g = torch.Generator().manual_seed(3)
    n, h = 2, 40
    x = torch.randn(n, 3, h, h, generator=g)
    wt = torch.randn(64, 3, 3, 3, generator=g) * 0.3
    b = torch.randn(64, generator=g)
    xr = H.nchw_to_nhwc(x.to(DEV), 4)
    wf, _ = H.pack_conv_weights(wt.to(DEV), 4)
    y = torch.ones(n * h * h, 64, device=DEV)
    H.conv_fwd(xr, None, wf, b.to(DEV), y, n, h, h, 64, 3, 1, 1, True, None)
    ref = F.conv2d(x, wt, b, padding=1) + 1.0
    assert rel(unrows(y, n, h, h), ref) < 2e-6
    dy = torch.randn(n, 64, h, h, generator=g)
    wg = wt.clone().requires_grad_(True)
    F.conv2d(x, wg, None, padding=1).backward(dy)
    dw = torch.empty(64, 3, 3, 3, device=DEV)
    H.conv_wgrad(rows(dy).to(DEV), xr, None, dw, n, h, h, 3, 1)
    assert rel(dw, wg.grad) < 2e-6


@pytest.mark.parametrize("c,n,h", [(16, 3, 10), (64, 3, 10), (512, 3, 10),
                                   # large enough that the kernels' four-rows-in-flight loops run
                                   (64, 40, 40), (512, 100, 10)])
def test_bn_relu_fwd_bwd(c, n, h):
    from superresolution_for_pdes_amd import hipops as H
    g = torch.Generator().manual_seed(c)
    y = torch.randn(n, c, h, h, generator=g) * 2 + 0.5
    gamma = torch.rand(c, generator=g) + 0.5
    beta = torch.randn(c, generator=g) * 0.2
    yv = y.clone().requires_grad_(True)
    gv = gamma.clone().requires_grad_(True)
    bv = beta.clone().requires_grad_(True)
    rm, rv = torch.zeros(c), torch.ones(c)
    a_ref = F.relu(F.batch_norm(yv, rm, rv, gv, bv, True, 0.1, 1e-5))
    da = torch.randn(n, c, h, h, generator=g)
    a_ref.backward(da)
    # HIP: stats via a 1x1 identity? use the exact batch stats path through finalize from partials
    yr = rows(y).to(DEV)
    P = n * h * h
    # build (mean, M2) partials of one block per 7 rows, exercising the Chan merge
    blk = 7
    nblk = (P + blk - 1) // blk
    st = torch.empty(nblk, c, 2, dtype=torch.float32)
    for k in range(nblk):
        seg = rows(y)[k * blk:(k + 1) * blk].double()
        st[k, :, 0] = seg.mean(0).float()
        st[k, :, 1] = ((seg - seg.mean(0)) ** 2).sum(0).float()
    rmd, rvd = torch.zeros(c, device=DEV), torch.ones(c, device=DEV)
    nbt = torch.zeros((), dtype=torch.int64, device=DEV)
    mean, invstd = H.bn_train_finalize(st.to(DEV), nblk, blk, P, rmd, rvd, nbt, 0.1, 1e-5)
    out = H.empty(P, c, device=DEV)
    H.bn_relu_fwd(yr, mean, invstd, gamma.to(DEV), beta.to(DEV), out)
    torch.cuda.synchronize()
    assert rel(unrows(out, n, h, h), a_ref) < 2e-6
    assert rel(rmd, rm) < 1e-6 and rel(rvd, rv) < 1e-6 and int(nbt) == 1
    dy = H.empty(P, c, device=DEV)
    dgam, dbet, dbias = (torch.empty(c, device=DEV) for _ in range(3))
    H.bn_relu_bwd(yr, rows(da).to(DEV), mean, invstd, gamma.to(DEV), beta.to(DEV), dy, dgam, dbet, dbias)
    torch.cuda.synchronize()
    assert rel(unrows(dy, n, h, h), yv.grad) < 1e-5
    assert rel(dgam, gv.grad) < 1e-5 and rel(dbet, bv.grad) < 1e-5
    assert abs(float(dbias.abs().max())) < 1e-3 * float(yv.grad.abs().max()) * P


def test_pool_upsample():
    from superresolution_for_pdes_amd import hipops as H
    g = torch.Generator().manual_seed(5)
    n, c, h = 2, 64, 20
    x = torch.randn(n, c, h, h, generator=g)
    x[:, :, 0, 0] = x[:, :, 0, 1]  # ties: first max wins
    xv = x.clone().requires_grad_(True)
    p_ref = F.max_pool2d(xv, 2)
    dp = torch.randn_like(p_ref)
    p_ref.backward(dp)
    xr = rows(x).to(DEV)
    p = H.maxpool_fwd(xr, n, h, h)
    dx = torch.full((n * h * h, c), 0.5, device=DEV)
    H.maxpool_bwd(xr, rows(dp).to(DEV), dx, n, h, h, True)
    torch.cuda.synchronize()
    assert torch.equal(unrows(p, n, h // 2, h // 2).cpu(), p_ref.detach())
    assert torch.allclose(unrows(dx, n, h, h).cpu(), xv.grad + 0.5)
    uv = x.clone().requires_grad_(True)
    u_ref = F.interpolate(uv, scale_factor=2, mode="bilinear", align_corners=True)
    du = torch.randn_like(u_ref)
    u_ref.backward(du)
    u = H.upsample_fwd(xr, n, h, h, 2 * h, 2 * h)
    dxu = H.empty(n * h * h, c, device=DEV)
    H.upsample_bwd(rows(du).to(DEV), dxu, n, h, h, 2 * h, 2 * h, False)
    torch.cuda.synchronize()
    assert rel(unrows(u, n, 2 * h, 2 * h), u_ref) < 1e-6
    assert rel(unrows(dxu, n, h, h), uv.grad) < 1e-6


@pytest.mark.parametrize("h,ho", [(20, 40), (10, 20), (7, 9), (2, 4), (5, 15), (4, 12)])
def test_upsample_bwd_gather_slots(h, ho):
    """The gather backward at the model's 2x ratios and at others up to the gather's cap (8
    candidates per axis) against torch's bilinear (align_corners=True) backward."""
    from superresolution_for_pdes_amd import hipops as H
    g = torch.Generator().manual_seed(h * 100 + ho)
    n, c = 2, 32
    x = torch.randn(n, c, h, h, generator=g).requires_grad_(True)
    u = F.interpolate(x, size=(ho, ho), mode="bilinear", align_corners=True)
    du = torch.randn(n, c, ho, ho, generator=g)
    u.backward(du)
    dx = H.empty(n * h * h, c, device=DEV)
    H.upsample_bwd(rows(du).to(DEV), dx, n, h, h, ho, ho, False)
    torch.cuda.synchronize()
    assert rel(unrows(dx, n, h, h), x.grad) < 1e-6


def test_upsample_bwd_rejects_ratios_beyond_the_gather_cap():
    from superresolution_for_pdes_amd import hipops as H
    dx = H.empty(2 * 3 * 3, 32, device=DEV)
    with pytest.raises(RuntimeError, match="ratio above 4"):
        H.upsample_bwd(torch.zeros(2 * 16 * 16, 32, device=DEV), dx, 2, 3, 3, 16, 16, False)


@pytest.mark.parametrize("c,h", [(128, 20), (256, 10)])
def test_upsample_bwd_with_gating_gradient(c, h):
    """upsample_bwd(gate=(dsa, wg)) == the upsample backward of dout + dsa (x) wg (the attention
    gating gradient, models.py:116, folded into its consumer, models.py:89/92)."""
    from superresolution_for_pdes_amd import hipops as H
    g = torch.Generator().manual_seed(11)
    n, ho = 3, 2 * h
    x = torch.randn(n, c, h, h, generator=g).requires_grad_(True)
    u = F.interpolate(x, scale_factor=2, mode="bilinear", align_corners=True)
    du = torch.randn(n, c, ho, ho, generator=g)
    dsa = torch.randn(n, 1, ho, ho, generator=g)
    wg = torch.randn(c, generator=g)
    u.backward(du + dsa * wg.view(1, c, 1, 1))
    dx = H.empty(n * h * h, c, device=DEV)
    H.upsample_bwd(rows(du).to(DEV), dx, n, h, h, ho, ho, False,
                   gate=(dsa.reshape(-1).contiguous().to(DEV), wg.to(DEV)))
    torch.cuda.synchronize()
    assert rel(unrows(dx, n, h, h), x.grad) < 1e-6


@pytest.mark.parametrize("c,gc,h", [(256, 512, 10), (64, 128, 40)])
def test_attention(c, gc, h):
    from superresolution_for_pdes_amd import hipops as H
    g = torch.Generator().manual_seed(c)
    n = 3
    x = torch.randn(n, c, h, h, generator=g)
    gt = torch.randn(n, gc, h, h, generator=g)
    w1 = torch.randn(c // 8, c, generator=g) * 0.2
    b1 = torch.randn(c // 8, generator=g) * 0.1
    w2 = torch.randn(c, c // 8, generator=g) * 0.2
    b2 = torch.randn(c, generator=g) * 0.1
    wg = torch.randn(1, gc, generator=g) * 0.1
    bg = torch.randn(1, generator=g) * 0.1
    # reference in fp64: fp32 CPU sums vary with the host's thread count at the 1e-5 level
    ts = [t.double().requires_grad_(True) for t in (x, gt, w1, b1, w2, b2, wg, bg)]
    xv, gv, w1v, b1v, w2v, b2v, wgv, bgv = ts
    m = xv.mean(dim=(2, 3), keepdim=True)
    hh = F.relu(F.conv2d(m, w1v[:, :, None, None], b1v))
    ca = torch.sigmoid(F.conv2d(hh, w2v[:, :, None, None], b2v))
    sa = torch.sigmoid(F.conv2d(gv, wgv[:, :, None, None], bgv))
    ref = xv * ca * sa
    dout = torch.randn(ref.shape, generator=g)
    ref.backward(dout.double())
    d = {k: v.to(DEV) for k, v in dict(w1=w1, b1=b1, w2=w2, b2=b2, wg=wg, bg=bg).items()}
    xr, gr = rows(x).to(DEV), rows(gt).to(DEV)
    out, saved = H.att_fwd(xr, gr, n, h * h, d["w1"], d["b1"], d["w2"], d["b2"], d["wg"], d["bg"])
    assert rel(unrows(out, n, h, h), ref) < 2e-6
    dx = H.empty(n * h * h, c, device=DEV)
    dg = torch.ones(n * h * h, gc, device=DEV)
    grads = [torch.empty_like(d[k]) for k in ("w1", "b1", "w2", "b2", "wg", "bg")]
    H.att_bwd(rows(dout).to(DEV), xr, gr, n, h * h, d["w1"], d["w2"], d["wg"], saved, dx, False, dg, True, *grads)
    torch.cuda.synchronize()
    assert rel(unrows(dx, n, h, h), xv.grad) < 1e-5
    assert rel(unrows(dg, n, h, h) - 1.0, gv.grad) < 1e-5
    for got, want in zip(grads, (w1v, b1v, w2v, b2v, wgv, bgv)):
        assert rel(got, want.grad) < 1e-5


def test_head_and_mse():
    from superresolution_for_pdes_amd import hipops as H
    g = torch.Generator().manual_seed(9)
    n, h = 3, 40
    z = torch.relu(torch.randn(n, 16, h, h, generator=g))
    xin = torch.randn(n, 3, h, h, generator=g)
    wf = torch.randn(1, 16, 1, 1, generator=g) * 0.3
    bf = torch.randn(1, generator=g)
    tgt = torch.randn(n, 1, h, h, generator=g)
    zv, wv, bv = (t.clone().requires_grad_(True) for t in (z, wf, bf))
    out_ref = F.conv2d(zv, wv, bv) + xin[:, 0:1]
    loss_ref = F.mse_loss(out_ref, tgt)
    loss_ref.backward()
    out = H.head_fwd(rows(z).to(DEV), wf.to(DEV), bf.to(DEV), xin.to(DEV), n, h * h)
    assert rel(out.view(n, 1, h, h), out_ref) < 1e-6
    loss = H.mse_fwd(out, tgt.to(DEV).view(-1))
    assert abs(float(loss) - float(loss_ref)) < 1e-5 * float(loss_ref)
    dy = H.mse_bwd(out, tgt.to(DEV).view(-1), None)
    dz = H.empty(n * h * h, 16, device=DEV)
    dwf, dbf = torch.empty(1, 16, 1, 1, device=DEV), torch.empty(1, device=DEV)
    H.head_bwd(dy, rows(z).to(DEV), wf.to(DEV), n, h * h, dz, dwf, dbf)
    torch.cuda.synchronize()
    assert rel(unrows(dz, n, h, h), zv.grad) < 1e-5
    assert rel(dwf, wv.grad) < 1e-5 and rel(dbf, bv.grad) < 1e-5


def test_clip_adamw_matches_torch():
    from superresolution_for_pdes_amd import hipops as H
    g = torch.Generator().manual_seed(1)
    ps = [torch.randn(1000, generator=g), torch.randn(37, generator=g)]
    gs = [torch.randn(1000, generator=g) * 3, torch.randn(37, generator=g)]
    ref = [torch.nn.Parameter(p.clone()) for p in ps]
    opt = torch.optim.AdamW(ref, lr=2e-4, weight_decay=1e-4)
    flat_p = torch.cat(ps).to(DEV)
    flat_g = torch.cat(gs).to(DEV)
    m = torch.zeros_like(flat_p)
    v = torch.zeros_like(flat_p)
    coef = torch.empty(2, device=DEV)
    for step in (1, 2, 3):
        for r, gg in zip(ref, gs):
            r.grad = gg.clone()
        tot = torch.nn.utils.clip_grad_norm_(ref, 1.0)
        opt.step()
        H.clip_coef(flat_g, 1.0, 1.0, coef)
        H.adamw_step(flat_p, flat_g, m, v, 2e-4, 0.9, 0.999, 1e-8, 1e-4, step, coef, 1.0)
        torch.cuda.synchronize()
        assert abs(float(coef[1]) - float(tot)) < 1e-5 * float(tot)
        assert rel(flat_p, torch.cat([r.detach() for r in ref])) < 1e-7


@pytest.mark.parametrize("scale", [1e-12, 1.0, 3e4])
def test_conv_h3_scale_invariance(scale, conv_math):
    """The h3 operand scales are powers of two picked from max|x|: scaling the input by any
    factor (tiny gradients, large activations) scales the output by the same factor with the
    same relative accuracy, and a loose max|x| upper bound (tag 1000x too big) changes nothing
    beyond rounding."""
    from superresolution_for_pdes_amd import hipops as H
    H.set_conv_math("h3")
    g = torch.Generator().manual_seed(11)
    n, cin, cout, h = 3, 128, 128, 20
    x = torch.randn(n, cin, h, h, generator=g, dtype=torch.float64) * scale
    wt = torch.randn(cout, cin, 3, 3, generator=g, dtype=torch.float64) * 0.03
    y64 = F.conv2d(x, wt, None, padding=1)
    xr = rows(x.float()).to(DEV)
    wf, _ = H.pack_conv_weights(wt.float().to(DEV), cin)
    y = H.empty(n * h * h, cout, device=DEV)
    H.conv_fwd(xr, None, wf, None, y, n, h, h, cout, 3, 1, 1, False, None)
    e_exact = rel(unrows(y, n, h, h), y64)
    loose = torch.tensor([int(np.float32(float(xr.abs().max()) * 1000).view(np.int32))], dtype=torch.int32, device=DEV)
    xr._srpde_amax = loose
    y2 = H.empty(n * h * h, cout, device=DEV)
    H.conv_fwd(xr, None, wf, None, y2, n, h, h, cout, 3, 1, 1, False, None)
    torch.cuda.synchronize()
    assert e_exact < 1e-6 and rel(unrows(y2, n, h, h), y64) < 1e-6, (e_exact, scale)


@pytest.mark.parametrize("log2_ratio", [6, 12, 18, 24])
def test_conv_h3_outlier_channel(log2_ratio, conv_math):
    """The h3 operand scale is per tensor: one channel 2^k larger than the rest sets it for all.
    Outputs that read only the small channels keep fp32-class accuracy while those channels sit
    within 2^-18 of the tensor's max (k <= 18: < 2e-6 relative); past that each small element keeps
    an absolute error <= 2^-40 of the max, i.e. a relative error growing as 2^(k-40)
    (k = 24: measured against that bound, not fp32's).  Outputs that read the outlier channel are
    dominated by it and stay exact to fp32 rounding."""
    from superresolution_for_pdes_amd import hipops as H
    H.set_conv_math("h3")
    g = torch.Generator().manual_seed(17 + log2_ratio)
    n, cin, cout, h = 2, 64, 64, 20
    x = torch.randn(n, cin, h, h, generator=g, dtype=torch.float64)
    x[:, 0] *= 2.0 ** log2_ratio
    wt = torch.randn(cout, cin, 3, 3, generator=g, dtype=torch.float64) * 0.05
    wt[: cout // 2, 0] = 0.0          # the first half of the outputs never reads the outlier channel
    y64 = F.conv2d(x, wt, None, padding=1)
    xr = rows(x.float()).to(DEV)
    wf, _ = H.pack_conv_weights(wt.float().to(DEV), cin)
    y = H.empty(n * h * h, cout, device=DEV)
    H.conv_fwd(xr, None, wf, None, y, n, h, h, cout, 3, 1, 1, False, None)
    torch.cuda.synchronize()
    yc = unrows(y, n, h, h)
    e_small = rel(yc[:, : cout // 2], y64[:, : cout // 2])
    e_big = rel(yc[:, cout // 2:], y64[:, cout // 2:])
    assert e_big < 2e-6, e_big
    if log2_ratio <= 18:
        assert e_small < 2e-6, e_small
    else:
        assert e_small < 4 * 2.0 ** (log2_ratio - 40) + 2e-6, e_small


def test_amax_words_match_outputs():
    """bn_relu_fwd / bn_relu_bwd write max|out| (float bits) into the word they are given."""
    from superresolution_for_pdes_amd import hipops as H
    g = torch.Generator().manual_seed(5)
    P, C = 5000, 64
    y = rows(torch.randn(1, C, 50, 100, generator=g)).to(DEV)
    mean, invstd = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    gam, bet = torch.rand(C, generator=g).to(DEV) + 0.5, torch.randn(C, generator=g).to(DEV)
    slots = H.AmaxSlots(2, DEV)
    out = H.empty(P, C, device=DEV)
    H.bn_relu_fwd(y, mean, invstd, gam, bet, out, amax=slots.take())
    dy = H.empty(P, C, device=DEV)
    da = rows(torch.randn(1, C, 50, 100, generator=g)).to(DEV)
    H.bn_relu_bwd(y, da, mean, invstd, gam, bet, dy, None, None, None, amax=slots.take())
    torch.cuda.synchronize()
    got = slots.buf.cpu().numpy().view(np.float32)
    assert got[0] == float(out.abs().max()) and got[1] == float(dy.abs().max())
    assert out._srpde_amax.data_ptr() == slots.buf.data_ptr()


@pytest.mark.parametrize("n,cin0,cin1,cout,h,dil", [
    (4, 512, 0, 512, 10, 2), (3, 512, 256, 256, 10, 1), (2, 256, 128, 128, 20, 1), (2, 128, 64, 64, 40, 1),
    (2, 64, 0, 32, 40, 1), (3, 64, 32, 96, 7, 2), (5, 128, 0, 128, 6, 1), (3, 64, 0, 64, 40, 1),
    (3, 64, 0, 64, 13, 2), (2, 64, 32, 32, 20, 1), (3, 32, 0, 16, 40, 1), (2, 32, 0, 16, 9, 1)])
def test_conv_wgrad_from_stored_splits(n, cin0, cin1, cout, h, dil, conv_math):
    """h3p: the forward and dgrad kernels store their operand splits (planes_out) and the weight
    gradient consumes them (no split work of its own).  Against fp64: within 3x the fp32-MFMA
    kernel's error (+1e-7) and < 1e-6 relative L2; ragged P, Cout not a tile multiple, dil 2 on 7x7.
    Cout = 16 (out_conv2): dy enters as 32-channel planes (zero channels 16..31, as
    srpde_bn_bwd_apply_split pads them) against the zero-padded dgrad weights; the dgrad is checked
    too."""
    from superresolution_for_pdes_amd import hipops as H
    g = torch.Generator().manual_seed(n * 31 + cout + cin0)
    cin = cin0 + cin1
    x = torch.randn(n, cin, h, h, generator=g, dtype=torch.float64)
    wt = torch.randn(cout, cin, 3, 3, generator=g, dtype=torch.float64) * (2.0 / (9 * cin)) ** 0.5
    dy = torch.randn(n, cout, h, h, generator=g, dtype=torch.float64) * 1e-3
    dw64 = torch.nn.grad.conv2d_weight(x, wt.shape, dy, padding=dil, dilation=dil)
    xr = rows(x.float()).to(DEV)
    x0, x1 = (xr[:, :cin0], xr[:, cin0:]) if cin1 else (xr, None)
    dyr = rows(dy.float()).to(DEV)
    P = n * h * h
    H.set_conv_math("h3")
    cp = H.cpad32(cout)
    assert H.h3_capable(cin0, cin1, cout, h, dil) and H.h3_capable(cp, 0, cin, h, dil)
    wf, wd = H.pack_conv_weights(wt.float().to(DEV), cin, want_dgrad=True)
    xp, dyp = H.split_planes_buffer(P, cin, DEV), H.split_planes_buffer(P, cp, DEV)
    y = H.empty(P, cout, device=DEV)
    H.conv_fwd(x0, x1, wf, None, y, n, h, h, cout, 3, dil, 1, False, None, xp)
    dx = H.empty(P, cin, device=DEV)
    dyin = dyr if cp == cout else torch.cat([dyr, torch.zeros(P, cp - cout, device=DEV)], 1)
    H.conv_fwd(dyin, None, wd, None, dx, n, h, h, cin, 3, dil, -1, False, None, dyp)
    if cp != cout:
        dx64 = torch.nn.grad.conv2d_input(x.shape, wt, dy, padding=dil, dilation=dil)
        assert rel(dx.view(n, h, h, cin).permute(0, 3, 1, 2).cpu(), dx64) < 1e-6
    dw = torch.empty(cout, cin, 3, 3, device=DEV)
    H.conv_wgrad_h3p(dyp, xp, dw, n, h, h, 3, dil)
    H.set_conv_math("f32")
    dwf = torch.empty(cout, cin, 3, 3, device=DEV)
    H.conv_wgrad(dyr, x0, x1, dwf, n, h, h, 3, dil)
    torch.cuda.synchronize()
    e_h3p, e_f32 = rel(dw, dw64), rel(dwf, dw64)
    print(f"wgrad h3p {e_h3p:.3e} f32 {e_f32:.3e}")
    assert e_h3p < 1e-6 and e_h3p < 3.0 * e_f32 + 1e-7, (e_h3p, e_f32)


def test_batched_weight_prep_matches_per_layer(conv_math):
    """srpde_prepare_weights_h3 (every layer's forward and dgrad planes in one launch) is
    bit-identical to pack + split per layer."""
    from superresolution_for_pdes_amd import hipops as H
    from superresolution_for_pdes_amd import unet_exec as X
    from superresolution_for_pdes_amd.models import UNet
    H.set_conv_math("h3")
    torch.manual_seed(0)
    m = UNet().to(DEV)
    X.prepare_h3_weights(m)
    checked = 0
    for name, c in m.named_modules():
        if not isinstance(c, torch.nn.Conv2d) or c.kernel_size != (3, 3):
            continue
        if c.in_channels % 4:   # enc1.conv1 (3 channels): no h3 packing either way
            assert c._srpde_h3f is None and c._srpde_h3d is None
            continue
        wf, wd = H.pack_conv_weights(c.weight.detach(), c.in_channels, want_fwd=True, want_dgrad=True)
        for got, ref in ((c._srpde_h3f, getattr(wf, "h3", None)), (c._srpde_h3d, getattr(wd, "h3", None))):
            assert (got is None) == (ref is None), name
            if got is not None:
                assert torch.equal(got.h3[0], ref[0]) and torch.equal(got.h3[1], ref[1]), name
                checked += 1
    assert checked >= 25, checked


@pytest.mark.parametrize("n,h,w", [(3, 40, 40), (2, 13, 7)])
def test_first_conv_direct_matches_fp64(n, h, w):
    """The 3-channel input conv (enc1.conv1: padded 4-float rows, 64 outputs): y against fp64
    (<= 1e-6 relative; the padding column meets zero weights) and the BN partials equal each
    256-row block's (mean, M2) of y itself (<= 1e-5 relative)."""
    from superresolution_for_pdes_amd import hipops as H
    g = torch.Generator().manual_seed(n + h)
    x = torch.randn(n, 3, h, w, generator=g, dtype=torch.float64)
    wt = torch.randn(64, 3, 3, 3, generator=g, dtype=torch.float64) * 0.3
    b = torch.randn(64, generator=g, dtype=torch.float64)
    ref = torch.nn.functional.conv2d(x, wt, b, padding=1)
    P = n * h * w
    x4 = torch.zeros(P, 4, dtype=torch.float32)
    x4[:, :3] = rows(x.float())
    x4[:, 3] = 7.0                       # padding column: must not contribute
    x4 = x4.to(DEV)
    wf = H.pack_conv_weights(wt.float().to(DEV), 4)[0]
    y = H.empty(P, 64, device=DEV)
    stats, nblk, rpb = H.conv_stats_buffer(n, h, w, 64, DEV, 4)
    H.conv_fwd(x4, None, wf, b.float().to(DEV), y, n, h, w, 64, 3, 1, 1, False, stats)
    torch.cuda.synchronize()
    yr = rows(ref)
    assert rel(y, yr) < 1e-6, rel(y, yr)
    yc = y.double().cpu()
    st = stats.double().cpu()
    for k in range(nblk):
        blk = yc[k * rpb:(k + 1) * rpb]
        mean = blk.mean(0)
        m2 = ((blk - mean) ** 2).sum(0)
        assert float((st[k, :, 0] - mean).abs().max()) <= 1e-5 * float(blk.abs().max())
        assert float((st[k, :, 1] - m2).abs().max()) <= 1e-5 * float(m2.abs().max()) + 1e-6


@pytest.mark.parametrize("n,h,w,c", [(3, 40, 40, 64), (2, 20, 6, 128)])
def test_bn_relu_pool_equals_separate_passes(n, h, w, c):
    """srpde_bn_relu_pool_fwd (a block output's BN + ReLU with its 2x2 max-pool in one pass) gives
    the same bits as srpde_bn_relu_fwd then srpde_maxpool2x2_fwd, ReLU-zero ties included, and the
    same max|out| word."""
    from superresolution_for_pdes_amd import hipops as H
    g = torch.Generator().manual_seed(c + h)
    P = n * h * w
    y = torch.randn(P, c, generator=g).to(DEV)
    mean, invstd = y.mean(0), 1.0 / torch.sqrt(y.var(0) + 1e-5)
    gam, bet = (torch.rand(c, generator=g) + 0.5).to(DEV), torch.randn(c, generator=g).to(DEV)
    slots = H.AmaxSlots(2, DEV)
    a1, a2 = H.empty(P, c, device=DEV), H.empty(P, c, device=DEV)
    H.bn_relu_fwd(y, mean, invstd, gam, bet, a1, amax=slots.take())
    p1 = H.maxpool_fwd(a1, n, h, w)
    p2 = H.empty(P // 4, c, device=DEV)
    H.bn_relu_pool_fwd(y, mean, invstd, gam, bet, a2, p2, n, h, w, amax=slots.take())
    torch.cuda.synchronize()
    assert torch.equal(a1, a2) and torch.equal(p1, p2)
    words = slots.buf.cpu()
    assert int(words[0]) == int(words[1])


@pytest.mark.parametrize("n,h,w,c", [(3, 40, 40, 64), (2, 20, 20, 128)])
def test_bn_relu_pool_att_matches_separate_passes(n, h, w, c):
    """srpde_bn_relu_pool_att_fwd: the activation and its pool bit-equal to srpde_bn_relu_pool_fwd, and
    the attention channel branch (m, h, ca) equal to srpde_att_channel_fwd of the activation to fp32
    summation order (<= 1e-6 relative)."""
    from superresolution_for_pdes_amd import hipops as H
    g = torch.Generator().manual_seed(c * 3 + h)
    P = n * h * w
    y = torch.randn(P, c, generator=g).to(DEV)
    mean, invstd = y.mean(0), 1.0 / torch.sqrt(y.var(0) + 1e-5)
    gam, bet = (torch.rand(c, generator=g) + 0.5).to(DEV), torch.randn(c, generator=g).to(DEV)
    w1 = (torch.randn(c // 8, c, generator=g) * 0.2).to(DEV)
    b1 = (torch.randn(c // 8, generator=g) * 0.1).to(DEV)
    w2 = (torch.randn(c, c // 8, generator=g) * 0.2).to(DEV)
    b2 = (torch.randn(c, generator=g) * 0.1).to(DEV)
    a1, a2 = H.empty(P, c, device=DEV), H.empty(P, c, device=DEV)
    p1, p2 = H.empty(P // 4, c, device=DEV), H.empty(P // 4, c, device=DEV)
    H.bn_relu_pool_fwd(y, mean, invstd, gam, bet, a1, p1, n, h, w)
    m1, h1, ca1 = H.att_channel_fwd(a1, n, h * w, w1, b1, w2, b2)
    m2, h2, ca2 = H.bn_relu_pool_att_fwd(y, mean, invstd, gam, bet, a2, p2, n, h, w, (w1, b1, w2, b2))
    torch.cuda.synchronize()
    assert torch.equal(a1, a2) and torch.equal(p1, p2)
    for u, v in ((m1, m2), (h1, h2), (ca1, ca2)):
        assert rel(v, u) < 1e-6, rel(v, u)


def test_bn_relu_att_unpooled_matches_separate_passes():
    """srpde_bn_relu_pool_att_fwd without a pool (enc3's output: 256 channels at 10x10): the activation
    bit-equal to srpde_bn_relu_fwd, the channel branch to fp32 summation order."""
    from superresolution_for_pdes_amd import hipops as H
    g = torch.Generator().manual_seed(11)
    n, h, w, c = 3, 10, 10, 256
    P = n * h * w
    y = torch.randn(P, c, generator=g).to(DEV)
    mean, invstd = y.mean(0), 1.0 / torch.sqrt(y.var(0) + 1e-5)
    gam, bet = (torch.rand(c, generator=g) + 0.5).to(DEV), torch.randn(c, generator=g).to(DEV)
    prm = tuple((torch.randn(*s, generator=g) * 0.2).to(DEV) for s in ((c // 8, c), (c // 8,), (c, c // 8), (c,)))
    a1, a2 = H.empty(P, c, device=DEV), H.empty(P, c, device=DEV)
    H.bn_relu_fwd(y, mean, invstd, gam, bet, a1)
    ref = H.att_channel_fwd(a1, n, h * w, *prm)
    got = H.bn_relu_pool_att_fwd(y, mean, invstd, gam, bet, a2, None, n, h, w, prm)
    torch.cuda.synchronize()
    assert torch.equal(a1, a2)
    for u, v in zip(ref, got):
        assert rel(v, u) < 1e-6, rel(v, u)


def test_bn_relu_gate_matches_separate_passes():
    """srpde_bn_relu_gate_fwd (the bridge output's BN + ReLU with att3's spatial attention): the
    activation bit-equal to srpde_bn_relu_fwd, sa to srpde_att_gate_fwd's within fp32 summation order."""
    from superresolution_for_pdes_amd import hipops as H
    g = torch.Generator().manual_seed(5)
    n, h, w, c = 3, 10, 10, 512
    P = n * h * w
    y = torch.randn(P, c, generator=g).to(DEV)
    mean, invstd = y.mean(0), 1.0 / torch.sqrt(y.var(0) + 1e-5)
    gam, bet = (torch.rand(c, generator=g) + 0.5).to(DEV), torch.randn(c, generator=g).to(DEV)
    wg, bg = (torch.randn(1, c, 1, 1, generator=g) * 0.05).to(DEV), torch.randn(1, generator=g).to(DEV)
    a1, a2 = H.empty(P, c, device=DEV), H.empty(P, c, device=DEV)
    H.bn_relu_fwd(y, mean, invstd, gam, bet, a1)
    x = torch.randn(P, 256, generator=g).to(DEV)
    chan = (torch.zeros(n, 256, device=DEV), torch.zeros(n, 32, device=DEV), torch.ones(n, 256, device=DEV))
    _, (_, _, _, sa_ref) = H.att_gate_fwd(x, a1, n, h * w, chan, wg, bg)
    sa = H.bn_relu_gate_fwd(y, mean, invstd, gam, bet, a2, wg, bg)
    torch.cuda.synchronize()
    assert torch.equal(a1, a2)
    assert float((sa - sa_ref).abs().max()) < 1e-6


@pytest.mark.parametrize("n,c,cout,hw,dil,sign", [(4, 64, 64, 40, 1, -1), (3, 128, 64, 20, 1, -1),
                                                  (2, 256, 512, 10, 2, -1), (4, 512, 256, 10, 1, -1),
                                                  (3, 64, 32, 40, 1, 1), (5, 128, 128, 20, 1, 1)])
def test_conv_presplit_equals_inline_split(n, c, cout, hw, dil, sign):
    """srpde_conv_fwd_h3_presplit on the split the inline kernel stored (planes_out) computes every
    output element, BN partial, fused BN-backward partial and per-tile max in equal bits: the same
    fp16 operands in the same MFMA order (8-wave kernel for >64 output channels, h3r below)."""
    from superresolution_for_pdes_amd import hipops as H
    H.set_conv_math("h3")
    g = torch.Generator(device=DEV).manual_seed(c + cout + hw)
    P = n * hw * hw
    x = torch.randn(P, c, device=DEV, generator=g)
    x._srpde_amax = H.amax_of(x)
    w = torch.randn(cout, c, 3, 3, device=DEV, generator=g) * 0.05
    b = torch.randn(cout, device=DEV, generator=g) if sign > 0 else None
    wf, _ = H.pack_conv_weights(w, c, True, False)   # [cout][tap][c] rows: either pass's layout
    by = torch.randn(P, cout, device=DEV, generator=g)
    bmean, binv = torch.randn(cout, device=DEV, generator=g) * 0.1, torch.rand(cout, device=DEV, generator=g) + 0.5
    bga, bbe = torch.randn(cout, device=DEV, generator=g), torch.randn(cout, device=DEV, generator=g) * 0.1
    outs = []
    xp = H.split_planes_buffer(P, c, DEV)
    for pre in (False, True):
        y = torch.empty(P, cout, device=DEV)
        part = H.bn_bwd_partials(n, hw, hw, cout, DEV)
        omax = H.out_max_slots(n, hw, hw, c, cout, dil, DEV)
        bnb = (by, bmean, binv, bga, bbe, part)
        if not pre:
            H.conv_fwd(x, None, wf, b, y, n, hw, hw, cout, 3, dil, sign, False, None, xp, bn_bwd=bnb, out_max=omax)
            xp._srpde_amax = x._srpde_amax
        else:
            H.conv_fwd_presplit(xp, wf, b, y, n, hw, hw, cout, 3, dil, sign, False, None, bn_bwd=bnb, out_max=omax)
        torch.cuda.synchronize()
        outs.append((y.clone(), part.clone(), omax.clone()))
    for name, a, b_ in zip(("y", "bn_part", "out_max"), *outs):
        assert torch.equal(a, b_), name


@pytest.mark.parametrize("P,C", [(1024 * 100, 256), (3 * 1600, 64), (777, 32), (2 * 1600 + 5, 16)])
def test_bn_bwd_apply_split_matches_fp32_apply(P, C):
    """srpde_bn_bwd_apply_split's planes hold bn_relu_bwd's dy: (hi + lo) / s equals the fp32 apply
    to the split's representation error (2^-22 of the scale), and the scale word is a bound.  C = 16
    (out_bn2): the planes are 32 channels wide, channels 16..31 exactly zero."""
    from superresolution_for_pdes_amd import hipops as H
    g = torch.Generator(device=DEV).manual_seed(P + C)
    y = torch.randn(P, C, device=DEV, generator=g) * 2 + 0.5
    da = torch.randn(P, C, device=DEV, generator=g)
    mean, invstd = y.mean(0), y.var(0, unbiased=False).add(1e-5).rsqrt()
    gamma = torch.randn(C, device=DEV, generator=g)
    beta = torch.randn(C, device=DEV, generator=g) * 0.1
    d1, d2, d3 = (torch.empty(C, device=DEV) for _ in range(3))
    m1, m2, word = H.bn_bwd_prepare(y, da, mean, invstd, gamma, beta, d1, d2, d3)
    planes = H.bn_bwd_apply_split(y, da, mean, invstd, gamma, beta, m1, m2, word)
    dy = torch.empty(P, C, device=DEV)
    e1, e2, e3 = (torch.empty(C, device=DEV) for _ in range(3))
    H.bn_relu_bwd(y, da, mean, invstd, gamma, beta, dy, e1, e2, e3)
    torch.cuda.synchronize()
    bound = float(word.view(torch.float32))
    assert bound >= float(dy.abs().max())
    e = int(np.floor(np.log2(bound))) + 1           # h3_exp: max < 2^e -> scale 2^(15 - e)
    s = 2.0 ** (15 - e)
    assert planes.shape == (2, P, H.cpad32(C))
    assert not bool(planes[:, :, C:].any())
    deq = (planes[0, :, :C].double() + planes[1, :, :C].double()) / s
    err = float((deq - dy.double()).abs().max())
    assert err <= 2.0 ** -22 * (2.0 ** 15 / s) + 1e-30, (err, bound)


@pytest.mark.parametrize("nblk,rpb,P,C", [
    (20480, 80, 1638400, 64),     # a 40x40 layer's h5 partials (80-row blocks)
    (20480, 80, 1638400, 16),     # out_bn2
    (3200, 128, 409600, 128),     # a 20x20 layer
    (800, 128, 102400, 512),      # a 10x10 layer
    (13, 7, 87, 48),              # ragged last block, C not a multiple of 16, fewer rows than one slice
    (1, 5, 3, 4),                 # one ragged block only (nfull = 0)
])
def test_bn_finalize_two_pass_matches_one_block_per_channel(nblk, rpb, P, C):
    """srpde_bn_train_finalize_ws (row slices of 16-channel groups, then the slices in order) against the
    one-block-per-channel kernel on the same (mean, M2) partials: mean / invstd / running statistics to
    fp32 rounding (the fp64 sums differ in order only), affine outputs and the max|a| bound word equal."""
    from superresolution_for_pdes_amd import hipops as H
    g = torch.Generator().manual_seed(nblk + C)
    st = torch.empty(nblk, C, 2)
    st[:, :, 0] = torch.randn(nblk, C, generator=g) * 0.3 + torch.linspace(-2, 2, C)
    st[:, :, 1] = torch.rand(nblk, C, generator=g) * rpb
    st = st.to(DEV)
    gam = (torch.rand(C, generator=g) + 0.5).to(DEV)
    bet = (torch.randn(C, generator=g) * 0.2).to(DEV)
    res = []
    saved = H._FIN_SPLIT, H._FIN_SPLIT_MIN_BLOCKS
    try:
        H._FIN_SPLIT_MIN_BLOCKS = 1   # the two-pass kernels at every size here
        for split in (False, True):
            H._FIN_SPLIT = split
            rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
            nbt = torch.zeros((), dtype=torch.int64, device=DEV)
            amax = torch.zeros(1, dtype=torch.int32, device=DEV)
            m, i, (sc, sh) = H.bn_train_finalize_affine(st, nblk, rpb, P, rm, rv, nbt, 0.1, 1e-5, gam, bet, amax=amax)
            m2, i2 = H.bn_train_finalize(st, nblk, rpb, P, None, None, None, 0.1, 1e-5)
            torch.cuda.synchronize()
            res.append((m, i, sc, sh, rm, rv, int(nbt), int(amax), m2, i2))
    finally:
        H._FIN_SPLIT, H._FIN_SPLIT_MIN_BLOCKS = saved
    a, b = res
    for k in (0, 1, 2, 3, 4, 5, 8, 9):
        assert torch.allclose(a[k], b[k], rtol=2e-7, atol=1e-7), (k, float((a[k] - b[k]).abs().max()))
    assert a[6] == b[6] == 1 and a[7] == b[7]
    assert torch.equal(b[0], b[8]) and torch.equal(b[1], b[9])   # the affine variant's mean / invstd are the plain one's
