"""The h5 convolution forward (conv_h5.hip: W = 40, tiles of 8 image rows, weight taps through an LDS ring) against the
h4 / h3r kernels it replaces for the U-Net's 40x40 layers (src/models.py:16,18,57: enc1.conv2, dec1.conv1,
dec1.conv2, out_conv1).  Same fragments, products, accumulation order and epilogue expressions, so the conv
outputs must be EQUAL bit for bit: plain, eval-mode epilogue (BN + ReLU, max|y| word), training (stored input
split, fused input BN + ReLU, gated second input).  The BN statistics come in 80-row blocks (h5) instead of
128-row ones: each set is checked against fp64 statistics of the same y, and the finalized batch statistics
of both agree to fp32 rounding."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _block_stats64(y, rows):
    """(mean, M2) per `rows`-row block of y [P, C] in fp64 (the conv epilogue's partial statistics)."""
    P, C = y.shape
    nb = -(-P // rows)
    out = torch.empty(nb, C, 2, dtype=torch.float64, device=y.device)
    yd = y.double()
    for b in range(nb):
        blk = yd[b * rows:(b + 1) * rows]
        m = blk.mean(0)
        out[b, :, 0] = m
        out[b, :, 1] = ((blk - m) ** 2).sum(0)
    return out


def _merged(stats, rows, P):
    """Chan-merge of (mean, M2) row blocks -> (mean, biased var) per channel, fp64."""
    s = stats.double()
    cnt = torch.full((s.shape[0],), float(rows), dtype=torch.float64, device=s.device)
    cnt[-1] = P - rows * (s.shape[0] - 1)
    n = cnt.sum()
    mean = (s[:, :, 0] * cnt[:, None]).sum(0) / n
    m2 = s[:, :, 1].sum(0) + (cnt[:, None] * (s[:, :, 0] - mean) ** 2).sum(0)
    return mean, m2 / n


@pytest.mark.parametrize("n,h,c0,c1,cout", [
    (5, 40, 64, 0, 64),      # enc1.conv2 / dec1.conv2 (fused input BN + ReLU in training)
    (3, 40, 128, 64, 64),    # dec1.conv1: [up(d2), att1(e1)] (virtual concat, gated second input)
    (4, 40, 64, 0, 32),      # out_conv1
    (2, 8, 64, 0, 64),       # one tile per sample: its top and bottom halo rows both outside
    (3, 16, 64, 64, 32),     # two tiles per sample, a plain concat
    (300, 40, 64, 0, 64),    # more tiles than CUs: persistent workgroups walk several tiles
])
def test_conv_h5_equals_h4(n, h, c0, c1, cout):
    from superresolution_for_pdes_amd import hipops as H
    if H.conv_math() != "h3":
        pytest.skip("h3 kernels off")
    w_ = 40
    cin = c0 + c1
    g = torch.Generator(device=DEV).manual_seed(17)
    P = n * h * w_
    x = torch.randn(P, cin, device=DEV, generator=g)
    x0, x1 = (x[:, :c0], x[:, c0:]) if c1 else (x, None)
    w = torch.randn(cout, cin, 3, 3, device=DEV, generator=g) * 0.05
    b = torch.randn(cout, device=DEV, generator=g)
    wf, _ = H.pack_conv_weights(w, cin, True, False)
    emean, einv = torch.randn(cout, device=DEV, generator=g) * 0.1, torch.rand(cout, device=DEV, generator=g) + 0.5
    ega, ebe = torch.randn(cout, device=DEV, generator=g), torch.randn(cout, device=DEV, generator=g) * 0.1
    for t in (x0, x1):
        if t is not None:
            t._srpde_amax = H.amax_of(t)
    aff = None
    gate = None
    if c1 == 0:
        aff = (torch.rand(c0, device=DEV, generator=g) + 0.5, torch.randn(c0, device=DEV, generator=g) * 0.2)
    elif c0 == 128:
        gate = (torch.sigmoid(torch.randn(n, c1, device=DEV, generator=g)),
                torch.sigmoid(torch.randn(P, device=DEV, generator=g)))
    outs = []
    prev = H.set_h5(True)
    try:
        for on in (False, True):
            H.set_h5(on)
            yp = torch.empty(P, cout, device=DEV)
            H.conv_fwd(x0, x1, wf, b, yp, n, h, w_, cout, 3, 1, 1, False, None)
            y = torch.empty(P, cout, device=DEV)
            stats, nblk, rows = H.conv_stats_buffer(n, h, w_, cout, DEV, c0, c1, 1)
            xp = H.split_planes_buffer(P, cin, DEV)
            H.conv_fwd(x0, x1, wf, b, y, n, h, w_, cout, 3, 1, 1, False, stats, xp, in_affine=aff, x1_gate=gate)
            ye = torch.empty(P, cout, device=DEV)
            eam = torch.zeros(1, dtype=torch.int32, device=DEV)
            H.conv_fwd(x0, x1, wf, b, ye, n, h, w_, cout, 3, 1, 1, False, None,
                       ep_bn=(emean, einv, ega, ebe, eam), x1_gate=gate)
            # the training paths in isolation: statistics without a stored split (the default at W = 40, whose
            # weight gradient splits the input itself -- round 5's null-pointer fault) and a split without statistics
            ys = torch.empty(P, cout, device=DEV)
            stats_s, _, _ = H.conv_stats_buffer(n, h, w_, cout, DEV, c0, c1, 1)
            H.conv_fwd(x0, x1, wf, b, ys, n, h, w_, cout, 3, 1, 1, False, stats_s, None, in_affine=aff, x1_gate=gate)
            yx = torch.empty(P, cout, device=DEV)
            xpx = H.split_planes_buffer(P, cin, DEV)
            H.conv_fwd(x0, x1, wf, b, yx, n, h, w_, cout, 3, 1, 1, False, None, xpx, in_affine=aff, x1_gate=gate)
            torch.cuda.synchronize()
            assert torch.equal(ys, y) and torch.equal(stats_s, stats), "statistics without a stored split"
            assert torch.equal(yx, y) and torch.equal(xpx, xp), "stored split without statistics"
            outs.append((yp, y, xp, ye, eam, stats, rows))
    finally:
        H.set_h5(prev)
    for name, a, b_ in zip(("y_plain", "y", "xsplit", "y_eval", "amax_eval"), outs[0][:5], outs[1][:5]):
        assert torch.equal(a, b_), name
    assert outs[1][6] == 80 and outs[0][6] == 128
    y = outs[1][1]
    for stats, rows in ((outs[0][5], outs[0][6]), (outs[1][5], outs[1][6])):
        ref = _block_stats64(y, rows)
        scale = float(ref[:, :, 1].abs().max()) + 1.0
        assert float((stats[:, :, 0].double() - ref[:, :, 0]).abs().max()) <= 1e-5 * (float(y.abs().max()) + 1)
        assert float((stats[:, :, 1].double() - ref[:, :, 1]).abs().max()) <= 1e-5 * scale
    m0, v0 = _merged(outs[0][5], outs[0][6], P)
    m1, v1 = _merged(outs[1][5], outs[1][6], P)
    assert float((m0 - m1).abs().max()) <= 1e-6 * (float(m0.abs().max()) + 1)
    assert float((v0 - v1).abs().max()) <= 1e-6 * float(v0.abs().max())


def test_conv_h5_accumulate_into_strided_output():
    """accumulate=1 into a channel slice of a wider output, a concat input with strided views."""
    from superresolution_for_pdes_amd import hipops as H
    n, h, c0, c1, cout = 2, 40, 64, 64, 64
    g = torch.Generator(device=DEV).manual_seed(23)
    P = n * h * 40
    big_in = torch.randn(P, 256, device=DEV, generator=g)
    x0, x1 = big_in[:, 0:c0], big_in[:, 128:128 + c1]
    w = torch.randn(cout, c0 + c1, 3, 3, device=DEV, generator=g) * 0.05
    wf, _ = H.pack_conv_weights(w, c0 + c1, True, False)
    x0._srpde_amax = H.amax_of(x0)
    x1._srpde_amax = H.amax_of(x1)
    base = torch.randn(P, 192, device=DEV, generator=g)
    outs = []
    prev = H.set_h5(True)
    try:
        for on in (False, True):
            H.set_h5(on)
            big = base.clone()
            H.conv_fwd(x0, x1, wf, None, big[:, 64:128], n, h, 40, cout, 3, 1, 1, True)
            torch.cuda.synchronize()
            outs.append(big)
    finally:
        H.set_h5(prev)
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("n,h", [(5, 40), (3, 16), (1, 7)])
def test_conv_n16_equals_h3r(n, h):
    """out_conv2's training forward (32 -> 16, conv_head.hip conv_fwd_n16_kernel) against the 32-column h3r
    tile it replaces: y and the stored input split bit for bit (same products, same order), the 128-row BN
    partials against fp64 statistics of the same y; with and without the fused input BN + ReLU; ragged
    last block (n * h * 40 % 128 != 0)."""
    from superresolution_for_pdes_amd import hipops as H
    if H.conv_math() != "h3":
        pytest.skip("h3 kernels off")
    w_, cin, cout = 40, 32, 16
    g = torch.Generator(device=DEV).manual_seed(23 + n)
    P = n * h * w_
    x = torch.randn(P, cin, device=DEV, generator=g)
    x._srpde_amax = H.amax_of(x)
    wt = torch.randn(cout, cin, 3, 3, device=DEV, generator=g) * 0.05
    b = torch.randn(cout, device=DEV, generator=g)
    wf, _ = H.pack_conv_weights(wt, cin, True, False)
    aff = (torch.rand(cin, device=DEV, generator=g) + 0.5, torch.randn(cin, device=DEV, generator=g) * 0.2)
    for in_aff in (None, aff):
        outs = []
        prev = H.set_h5(True)
        try:
            for on in (False, True):
                H.set_h5(on)
                y = torch.empty(P, cout, device=DEV)
                stats, nblk, rows = H.conv_stats_buffer(n, h, w_, cout, DEV, cin, 0, 1)
                xp = H.split_planes_buffer(P, cin, DEV)
                H.conv_fwd(x, None, wf, b, y, n, h, w_, cout, 3, 1, 1, False, stats, xp, in_affine=in_aff)
                torch.cuda.synchronize()
                outs.append((y, xp, stats, rows))
        finally:
            H.set_h5(prev)
        assert torch.equal(outs[0][0], outs[1][0]), "y"
        assert torch.equal(outs[0][1], outs[1][1]), "xsplit"
        y, _, stats, rows = outs[1]
        assert rows == 128
        ref = _block_stats64(y, rows)
        got = stats.double().view(ref.shape)
        assert torch.allclose(got[:, :, 0], ref[:, :, 0], rtol=1e-5, atol=1e-6)
        assert torch.allclose(got[:, :, 1], ref[:, :, 1], rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("n", [3, 300])
def test_conv_h5_upsampled_input_equals_h4(n):
    """The eval decoder's dec1.conv1 on h5 (x0 = the bilinear x2 upsample of d, interpolated in h5's convert,
    one unit per tap; x1 gated; BN + ReLU epilogue) against the materialised upsample through h5 (output and
    max word bit for bit) and against h4's upsampled-input kernel."""
    from superresolution_for_pdes_amd import hipops as H
    if H.conv_math() != "h3":
        pytest.skip("h3 kernels off")
    g = torch.Generator(device=DEV).manual_seed(31)
    hw, hl, c0, c1, cout = 40, 20, 128, 64, 64
    d = torch.randn(n * hl * hl, c0, device=DEV, generator=g)
    e = torch.randn(n * hw * hw, c1, device=DEV, generator=g)
    ca = torch.sigmoid(torch.randn(n, c1, device=DEV, generator=g))
    w = torch.randn(cout, c0 + c1, 3, 3, device=DEV, generator=g) * 0.05
    b = torch.randn(cout, device=DEV, generator=g)
    wf, _ = H.pack_conv_weights(w, c0 + c1, True, False)
    wg = torch.randn(1, c0, 1, 1, device=DEV, generator=g) * 0.1
    bg = torch.randn(1, device=DEV, generator=g)
    emean, einv = torch.randn(cout, device=DEV, generator=g) * 0.1, torch.rand(cout, device=DEV, generator=g) + 0.5
    ega, ebe = torch.randn(cout, device=DEV, generator=g), torch.randn(cout, device=DEV, generator=g) * 0.1
    d._srpde_amax = H.amax_of(d)
    e._srpde_amax = H.amax_of(e)
    u, sa = H.upsample_gate_fwd(d, n, hl, hl, hw, hw, wg, bg)
    P = n * hw * hw
    outs = []
    prev = H.set_h5(True)
    try:
        for on, x0 in ((True, H.UpsampledInput(d, n, hl, hl)), (False, H.UpsampledInput(d, n, hl, hl)), (True, u)):
            H.set_h5(on)
            ye = torch.empty(P, cout, device=DEV)
            eam = torch.zeros(1, dtype=torch.int32, device=DEV)
            H.conv_fwd(x0, e, wf, b, ye, n, hw, hw, cout, 3, 1, 1, False, None, ep_bn=(emean, einv, ega, ebe, eam),
                       x1_gate=(ca, sa))
            torch.cuda.synchronize()
            outs.append((ye, eam))
    finally:
        H.set_h5(prev)
    # the materialised upsample through h5: bit for bit
    assert torch.equal(outs[0][0], outs[2][0]) and torch.equal(outs[0][1], outs[2][1])
    # h4's upsampled-input kernel: bit for bit where it runs whole tiles; with more tiles than CUs its last
    # tiles are K-split (summed by conv_tail_fixup in another order), so there fp32 rounding apart
    if n * hw * hw <= 256 * 256:
        assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    else:
        torch.testing.assert_close(outs[0][0], outs[1][0], rtol=1e-5, atol=1e-5)
