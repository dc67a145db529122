"""The h4 convolution kernel (conv_h4.hip) against the h3 kernels it replaces (the 8-wave kernel for
W = 10 (dilation 1 and 2) and W = 20, the 4-wave h3r for the 64-column tiles at W = 40): same fragments, products, accumulation order and
epilogue, so every output must be EQUAL bit for bit -- forward (bias, BN statistics, stored input
split, fused input BN + ReLU, virtual concat, the K-split tail), the eval-mode epilogue (BN + ReLU,
max|y| word), the dgrad from an fp32 dy (stored dy split, fused BN-backward partials, per-tile
max|dx|) and the dgrad from a pre-split dy.  The layer shapes are the U-Net's
(src/models.py:16-19, 43-49: enc1 / dec1 at 40x40, enc2 / dec2 at 20x20, enc3 / bridge / dec3 at 10x10)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("n,c0,c1,cout,hw,dil", [
    (9, 128, 0, 128, 20, 1),      # enc2.conv2 / dec2.conv2 (fused input BN + ReLU)
    (7, 256, 128, 128, 20, 1),    # dec2.conv1 (virtual concat)
    (21, 128, 0, 256, 10, 1),     # enc3.conv1
    (13, 512, 256, 256, 10, 1),   # dec3.conv1 (virtual concat)
    (11, 256, 0, 512, 10, 2),     # bridge.0
    (170, 512, 0, 512, 10, 2),    # bridge.3 with a K-split tail (268 tiles on 256 CUs)
    (2, 64, 64, 128, 20, 1),      # a partial last row tile, two 32-channel chunks per input
    # 64-column tiles (h3: the 4-wave h3r kernel at W = 40, the 8-wave kernel below)
    (5, 64, 0, 64, 40, 1),        # enc1.conv2 / dec1.conv2 (fused input BN + ReLU; dgrad 64 columns)
    (3, 128, 64, 64, 40, 1),      # dec1.conv1 (virtual concat; dgrad 192 columns = 3 tiles)
    (44, 64, 0, 64, 40, 1),       # W = 40 with a K-split tail (275 tiles; h3r has none: see below)
    (9, 64, 0, 128, 20, 1),       # enc2.conv1 (dgrad: 64 columns at W = 20)
    (6, 64, 0, 64, 10, 2),        # 64 columns at W = 10, dilation 2
])
def test_conv_h4_equals_h3(n, c0, c1, cout, hw, dil):
    from superresolution_for_pdes_amd import hipops as H
    if H.conv_math() != "h3":
        pytest.skip("h3 kernels off")
    cin = c0 + c1
    g = torch.Generator(device=DEV).manual_seed(7)
    P = n * hw * hw
    x = torch.randn(P, cin, device=DEV, generator=g)
    x0, x1 = (x[:, :c0], x[:, c0:]) if c1 else (x, None)
    w = torch.randn(cout, cin, 3, 3, device=DEV, generator=g) * 0.05
    b = torch.randn(cout, device=DEV, generator=g)
    wf, wd = H.pack_conv_weights(w, cin, True, True)
    dy = torch.randn(P, cout, device=DEV, generator=g)
    by = torch.randn(P, cin, device=DEV, generator=g)
    bmean, binv = torch.randn(cin, device=DEV, generator=g) * 0.1, torch.rand(cin, device=DEV, generator=g) + 0.5
    bga, bbe = torch.randn(cin, device=DEV, generator=g), torch.randn(cin, device=DEV, generator=g) * 0.1
    emean, einv = torch.randn(cout, device=DEV, generator=g) * 0.1, torch.rand(cout, device=DEV, generator=g) + 0.5
    ega, ebe = torch.randn(cout, device=DEV, generator=g), torch.randn(cout, device=DEV, generator=g) * 0.1
    for t in (x0, x1, dy):
        if t is not None:
            t._srpde_amax = H.amax_of(t)
    aff = None
    if c1 == 0:
        aff = (torch.rand(c0, device=DEV, generator=g) + 0.5, torch.randn(c0, device=DEV, generator=g) * 0.2)
    outs = []
    prev = H.set_h4(True)
    try:
        for on in (False, True):
            H.set_h4(on)
            y = torch.empty(P, cout, device=DEV)
            stats, _, _ = H.conv_stats_buffer(n, hw, hw, cout, DEV, c0, c1, dil)
            xp = H.split_planes_buffer(P, cin, DEV)
            H.conv_fwd(x0, x1, wf, b, y, n, hw, hw, cout, 3, dil, 1, False, stats, xp, in_affine=aff)
            ye = torch.empty(P, cout, device=DEV)
            eam = torch.zeros(1, dtype=torch.int32, device=DEV)
            H.conv_fwd(x0, x1, wf, b, ye, n, hw, hw, cout, 3, dil, 1, False, None, ep_bn=(emean, einv, ega, ebe, eam))
            dx = torch.empty(P, cin, device=DEV)
            dyp = H.split_planes_buffer(P, cout, DEV)
            part = H.bn_bwd_partials(n, hw, hw, cin, DEV)
            dmax = H.out_max_slots(n, hw, hw, cout, cin, dil, DEV)
            H.conv_fwd(dy, None, wd, None, dx, n, hw, hw, cin, 3, dil, -1, False, None, dyp,
                       bn_bwd=(by, bmean, binv, bga, bbe, part), out_max=dmax)
            dx2 = torch.empty(P, cin, device=DEV)
            part2 = H.bn_bwd_partials(n, hw, hw, cin, DEV)
            dmax2 = H.out_max_slots(n, hw, hw, cout, cin, dil, DEV)
            H.conv_fwd_presplit(dyp, wd, None, dx2, n, hw, hw, cin, 3, dil, -1, False, None,
                                bn_bwd=(by, bmean, binv, bga, bbe, part2), out_max=dmax2)
            torch.cuda.synchronize()
            outs.append((y, stats, xp, ye, eam, dx, dyp, part, dmax, dx2, part2, dmax2))
    finally:
        H.set_h4(prev)
    names = ("y", "stats", "xsplit", "y_eval", "amax_eval", "dx", "dysplit", "bn_part", "dx_max", "dx_presplit",
             "bn_part_presplit", "dx_max_presplit")
    for name, a, b_ in zip(names, *outs):
        if (name == "stats" or name.startswith("bn_part")) and hw == 40 and n == 44:
            # h3r runs no K-split tail: its last-round tiles' reductions are summed in another order
            # than conv_tail_fixup's (same y bits; statistics equal to fp32 rounding)
            assert float((a - b_).abs().max()) <= 1e-6 * float(b_.abs().max()), name
            continue
        assert torch.equal(a, b_), name
    # the pre-split dgrad reads the same pieces the fp32 one split: equal outputs as well
    assert torch.equal(outs[1][5], outs[1][9])


def test_conv_h4_accumulate_and_strided_output():
    """accumulate=1 into a channel slice of a wider output (the dgrad into a virtual-concat input)."""
    from superresolution_for_pdes_amd import hipops as H
    n, cin, cout, hw = 6, 256, 128, 10
    g = torch.Generator(device=DEV).manual_seed(3)
    P = n * hw * hw
    dy = torch.randn(P, cout, device=DEV, generator=g)
    w = torch.randn(cout, cin, 3, 3, device=DEV, generator=g) * 0.05
    _, wd = H.pack_conv_weights(w, cin, True, True)
    dy._srpde_amax = H.amax_of(dy)
    base = torch.randn(P, cin + 128, device=DEV, generator=g)
    outs = []
    prev = H.set_h4(True)
    try:
        for on in (False, True):
            H.set_h4(on)
            big = base.clone()
            H.conv_fwd(dy, None, wd, None, big[:, 64:64 + cin], n, hw, hw, cin, 3, 1, -1, True)
            torch.cuda.synchronize()
            outs.append(big)
    finally:
        H.set_h4(prev)
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("n,c0,c1,cout,hw,h4", [
    (13, 512, 256, 256, 10, True),    # dec3.conv1: [b, att3(e3)] on h4
    (7, 256, 128, 128, 20, True),     # dec2.conv1: [up(d3), att2(e2)] on h4
    (13, 512, 256, 256, 10, False),   # the same on the h3 8-wave kernel
    (3, 128, 64, 64, 40, True),       # dec1.conv1: [up(d2), att1(e1)] on h4 (64-column tiles)
    (3, 128, 64, 64, 40, False),      # the same on h3r
])
def test_gated_second_input_equals_materialized(n, c0, c1, cout, hw, h4):
    """The decoder conv reading an AttentionGate's output through x1_gate (the gate (x * ca) * sa
    formed in the operand transform, models.py:119-130) equals, bit for bit, the same conv reading the
    tensor srpde_att_apply_fwd writes: output, BN statistics, stored input split, and the eval-mode
    epilogue's output and max word."""
    from superresolution_for_pdes_amd import hipops as H
    cin = c0 + c1
    g = torch.Generator(device=DEV).manual_seed(11)
    P = n * hw * hw
    x0 = torch.randn(P, c0, device=DEV, generator=g)
    e = torch.randn(P, c1, device=DEV, generator=g)
    ca = torch.sigmoid(torch.randn(n, c1, device=DEV, generator=g))
    sa = torch.sigmoid(torch.randn(P, device=DEV, generator=g))
    w = torch.randn(cout, cin, 3, 3, device=DEV, generator=g) * 0.05
    b = torch.randn(cout, device=DEV, generator=g)
    wf, _ = H.pack_conv_weights(w, cin, True, False)
    emean, einv = torch.randn(cout, device=DEV, generator=g) * 0.1, torch.rand(cout, device=DEV, generator=g) + 0.5
    ega, ebe = torch.randn(cout, device=DEV, generator=g), torch.randn(cout, device=DEV, generator=g) * 0.1
    x0._srpde_amax = H.amax_of(x0)
    e._srpde_amax = H.amax_of(e)
    ea, _ = H.att_apply_fwd(e, n, hw * hw, (None, None, ca), sa)   # carries e's max word, as in the model
    outs = []
    prev = H.set_h4(h4)
    try:
        for x1, gate in ((ea, None), (e, (ca, sa))):
            y = torch.empty(P, cout, device=DEV)
            stats, _, _ = H.conv_stats_buffer(n, hw, hw, cout, DEV, c0, c1, 1)
            xp = H.split_planes_buffer(P, cin, DEV)
            H.conv_fwd(x0, x1, wf, b, y, n, hw, hw, cout, 3, 1, 1, False, stats, xp, x1_gate=gate)
            ye = torch.empty(P, cout, device=DEV)
            eam = torch.zeros(1, dtype=torch.int32, device=DEV)
            H.conv_fwd(x0, x1, wf, b, ye, n, hw, hw, cout, 3, 1, 1, False, None,
                       ep_bn=(emean, einv, ega, ebe, eam), x1_gate=gate)
            torch.cuda.synchronize()
            outs.append((y, stats, xp, ye, eam))
    finally:
        H.set_h4(prev)
    for name, a, b_ in zip(("y", "stats", "xsplit", "y_eval", "amax_eval"), *outs):
        assert torch.equal(a, b_), name


@pytest.mark.parametrize("n,c0,c1,cout,hw", [
    (9, 256, 128, 128, 20),    # dec2.conv1: [up(d3), att2(e2)]
    (5, 128, 64, 64, 40),      # dec1.conv1: [up(d2), att1(e1)]
    (44, 128, 64, 64, 40),     # many tiles per persistent workgroup, image boundaries inside tiles
])
def test_upsampled_input_equals_materialized(n, c0, c1, cout, hw):
    """The decoder conv reading up(d) through x0_up (the bilinear x2 upsample formed in the operand
    transform from d's low-res rows, models.py:70,89,92) equals, bit for bit, the same conv reading
    the tensor srpde_upsample_bilinear_fwd writes (same operand scale: the source's max word): output,
    BN statistics, stored input split, eval epilogue output and max word.  The gate's spatial attention
    from d at low resolution (srpde_upsample_gate_sa) equals the materialised form's to fp32 rounding."""
    from superresolution_for_pdes_amd import hipops as H
    g = torch.Generator(device=DEV).manual_seed(5)
    hl = hw // 2
    d = torch.randn(n * hl * hl, c0, device=DEV, generator=g)
    e = torch.randn(n * hw * hw, c1, device=DEV, generator=g)
    ca = torch.sigmoid(torch.randn(n, c1, device=DEV, generator=g))
    cin = c0 + c1
    w = torch.randn(cout, cin, 3, 3, device=DEV, generator=g) * 0.05
    b = torch.randn(cout, device=DEV, generator=g)
    wf, _ = H.pack_conv_weights(w, cin, True, False)
    wg = torch.randn(1, c0, 1, 1, device=DEV, generator=g) * 0.1
    bg = torch.randn(1, device=DEV, generator=g)
    emean, einv = torch.randn(cout, device=DEV, generator=g) * 0.1, torch.rand(cout, device=DEV, generator=g) + 0.5
    ega, ebe = torch.randn(cout, device=DEV, generator=g), torch.randn(cout, device=DEV, generator=g) * 0.1
    d._srpde_amax = H.amax_of(d)
    e._srpde_amax = H.amax_of(e)
    u, sa_ref = H.upsample_gate_fwd(d, n, hl, hl, hw, hw, wg, bg)
    sa = H.upsample_gate_sa(d, n, hl, hl, hw, hw, wg, bg)
    P = n * hw * hw
    prev = H.set_h4(True)
    outs = []
    try:
        for x0 in (u, H.UpsampledInput(d, n, hl, hl)):
            y = torch.empty(P, cout, device=DEV)
            stats, _, _ = H.conv_stats_buffer(n, hw, hw, cout, DEV, c0, c1, 1)
            xp = H.split_planes_buffer(P, cin, DEV)
            H.conv_fwd(x0, e, wf, b, y, n, hw, hw, cout, 3, 1, 1, False, stats, xp, x1_gate=(ca, sa_ref))
            ye = torch.empty(P, cout, device=DEV)
            eam = torch.zeros(1, dtype=torch.int32, device=DEV)
            H.conv_fwd(x0, e, wf, b, ye, n, hw, hw, cout, 3, 1, 1, False, None, ep_bn=(emean, einv, ega, ebe, eam),
                       x1_gate=(ca, sa_ref))
            torch.cuda.synchronize()
            outs.append((y, stats, xp, ye, eam))
    finally:
        H.set_h4(prev)
    for name, a, b_ in zip(("y", "stats", "xsplit", "y_eval", "amax_eval"), *outs):
        assert torch.equal(a, b_), name
    assert float((sa - sa_ref).abs().max()) <= 1e-6, float((sa - sa_ref).abs().max())
