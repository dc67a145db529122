"""Pointwise kernels stay bit-repeatable while MFMA convolutions run beside them on another stream.

The training step runs weight gradients on a side stream (unet_exec.WgradStream) concurrently with
the main stream's BN / upsample / gate passes.  On the MI355X boxes, packed-FP32 VALU instructions
(v_pk_fma/mul/add_f32) gave wrong lanes 48-63 under exactly that overlap, so the library is built
without them (build.py NO_PK); this is the end-to-end guard: each main-stream result
must equal the one computed with the GPU otherwise idle."""
import pytest
import torch

from superresolution_for_pdes_amd import hipops as H

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _conv_load(g):
    n, hw, c = 64, 20, 256
    x = torch.randn(n * hw * hw, c, device=DEV, generator=g).abs()
    x._srpde_amax = H.amax_of(x)
    wf, _ = H.pack_conv_weights(torch.randn(c, c, 3, 3, device=DEV, generator=g) * 0.05, c, True, False)
    b = torch.zeros(c, device=DEV)
    y = torch.empty(n * hw * hw, c, device=DEV)

    def run():
        for _ in range(6):
            H.conv_fwd(x, None, wf, b, y, n, hw, hw, c, 3, 1, 1, False, None)
    return run


def test_pointwise_repeatable_beside_side_stream_convs():
    torch.cuda.set_device(DEV)
    g = torch.Generator(device=DEV).manual_seed(7)
    n, h, w, c = 64, 20, 20, 128
    y = torch.randn(n * h * w, c, device=DEV, generator=g)
    mean, invstd = torch.randn(c, device=DEV, generator=g) * 0.1, torch.rand(c, device=DEV, generator=g) + 0.5
    gam, bet = torch.rand(c, device=DEV, generator=g) + 0.5, torch.randn(c, device=DEV, generator=g) * 0.1
    wg, bg = torch.randn(c, device=DEV, generator=g) * 0.1, torch.zeros(1, device=DEV)
    load = _conv_load(g)

    def victim():
        a = H.empty(n * h * w, c, device=DEV)
        H.bn_relu_fwd(y, mean, invstd, gam, bet, a, amax=None)
        u, sa = H.upsample_gate_fwd(a, n, h, w, 2 * h, 2 * w, wg, bg)
        return a, u, sa

    ref = [t.clone() for t in victim()]
    torch.cuda.synchronize()
    side = torch.cuda.Stream(DEV)
    bad = 0
    for _ in range(60):
        side.wait_stream(torch.cuda.current_stream(DEV))
        with torch.cuda.stream(side):
            load()
        out = victim()
        torch.cuda.current_stream(DEV).wait_stream(side)
        torch.cuda.synchronize()
        bad += not all(torch.equal(a, b) for a, b in zip(ref, out))
    assert bad == 0, f"{bad}/60 repeats differ"
