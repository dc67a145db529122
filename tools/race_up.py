"""Is upsample_gate_fwd (pointwise.hip) itself unrepeatable while another process runs the U-Net
forward on the same GPU?  rank 0: bn_relu_fwd -> upsample_gate_fwd -> upsample_gate_fwd again on the
same input, each output compared with the first iteration's; rank 1: the train forward as load."""
import ctypes
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from superresolution_for_pdes_amd import hipops as H  # noqa: E402
from superresolution_for_pdes_amd import unet_exec as X  # noqa: E402
from superresolution_for_pdes_amd.models import UNet, init_weights  # noqa: E402

DEV = torch.device("cuda", 0)
rank = int(os.environ.get("RANK", "0"))
NOISE_MODES = {"perm": 3, "mfma16": 4, "mfma32": 5, "mfma16k16": 6, "mfma32k8": 7, "mfma16f32": 8, "mfma16bf": 9}


def main():
    torch.cuda.set_device(DEV)
    torch.manual_seed(42)
    if rank > 0:
        noise = os.environ.get("NOISE", "fwd")
        m = UNet()
        m.apply(init_weights)
        m = m.to(DEV).train()
        x = torch.randn(64, 3, 40, 40, device=DEV)
        t_end = time.time() + float(os.environ.get("NOISE_S", "60"))
        convs = []
        for c, hw, h3r in ((128, 20, False), (64, 40, True)):
            xc = torch.randn(64 * hw * hw, c, device=DEV).abs()
            xc._srpde_amax = H.amax_of(xc)
            wf, _ = H.pack_conv_weights(torch.randn(c, c, 3, 3, device=DEV) * 0.05, c, True, False)
            convs.append((c, hw, h3r, xc, wf, torch.zeros(c, device=DEV)))
        big = torch.zeros(1 << 27, device=DEV)
        VICN = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "gpu", "lib", "libvictim.so"))
        ua = torch.rand(64 * 400, 128, device=DEV)
        wg0, bg0 = torch.randn(128, device=DEV), torch.zeros(1, device=DEV)
        with torch.no_grad():
            while time.time() < t_end:
                if noise == "fwd":
                    X.unet_forward(m, x, True, save=True)
                elif noise == "conv":
                    for c, hw, h3r, xc, wf, b in convs:
                        H.set_h3r(h3r)
                        y = torch.empty(64 * hw * hw, c, device=DEV)
                        st, _, _ = H.conv_stats_buffer(64, hw, hw, c, DEV, c, 0, 1)
                        xp = H.split_planes_buffer(64 * hw * hw, c, DEV)
                        H.conv_fwd(xc, None, wf, b, y, 64, hw, hw, c, 3, 1, 1, False, st, xp)
                elif noise.startswith("dma"):
                    md = {"dma_in": 0, "dma_oob": 1, "dma_plain": 2}[noise]
                    assert VICN.dma_noise(md, ctypes.c_void_p(big.data_ptr()), ctypes.c_uint(1 << 28), 4096, 400,
                                          ctypes.c_void_p(big.data_ptr()), ctypes.c_void_p(H.stream_ptr())) == 0
                elif noise in NOISE_MODES:
                    assert VICN.valu_noise(NOISE_MODES[noise], 4096, 20000, ctypes.c_void_p(big.data_ptr()),
                                           ctypes.c_void_p(H.stream_ptr())) == 0
                elif noise == "upgate":
                    H.upsample_gate_fwd(ua, 64, 20, 20, 40, 40, wg0, bg0)
                else:
                    big.mul_(1.0001)
                torch.cuda.synchronize()
        print(f"rank {rank} noise done", flush=True)
        return
    mode = os.environ.get("UPMODE", "gate")
    global VIC
    if mode.startswith("k"):
        VIC = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "gpu", "lib",
                                       os.environ.get("VICLIB", "libvictim.so")))
    intra = os.environ.get("INTRA", "")   # one process: this noise kernel on a second stream beside each rep
    side = torch.cuda.Stream(DEV)
    junk = torch.zeros(16, device=DEV)
    n, h, w, c = 64, 20, 20, 128
    y = torch.randn(n * h * w, c, device=DEV)
    mean, invstd = torch.randn(c, device=DEV) * 0.1, torch.rand(c, device=DEV) + 0.5
    gam, bet = torch.rand(c, device=DEV) + 0.5, torch.randn(c, device=DEV) * 0.1
    wg, bg = torch.randn(c, device=DEV) * 0.1, torch.zeros(1, device=DEV)
    ref = None
    bad = [0, 0, 0]
    reps = int(os.environ.get("STRESS_REPS", "400"))
    for k in range(reps):
        if intra:
            side.wait_stream(torch.cuda.current_stream(DEV))
            with torch.cuda.stream(side):
                assert VIC.valu_noise(NOISE_MODES[intra], 2048, 20000, ctypes.c_void_p(junk.data_ptr()),
                                      ctypes.c_void_p(H.stream_ptr())) == 0
        a = H.empty(n * h * w, c, device=DEV)
        H.bn_relu_fwd(y, mean, invstd, gam, bet, a, amax=None)
        if mode.startswith("k"):
            u1, s1 = torch.empty(n * 4 * h * w, c, device=DEV), torch.empty(n * 4 * h * w, device=DEV)
            u2, s2 = torch.empty_like(u1), torch.empty_like(s1)
            for u, sv in ((u1, s1), (u2, s2)):
                rc = VIC.victim_upsample_gate(int(mode[1:]), ctypes.c_void_p(a.data_ptr()), ctypes.c_void_p(u.data_ptr()),
                                              n, h, w, c, ctypes.c_void_p(wg.data_ptr()), ctypes.c_void_p(bg.data_ptr()),
                                              ctypes.c_void_p(sv.data_ptr()), ctypes.c_void_p(H.stream_ptr()))
                assert rc == 0
        elif mode == "gate":
            u1, s1 = H.upsample_gate_fwd(a, n, h, w, 2 * h, 2 * w, wg, bg)
            u2, s2 = H.upsample_gate_fwd(a, n, h, w, 2 * h, 2 * w, wg, bg)
        else:
            u1 = H.upsample_fwd(a, n, h, w, 2 * h, 2 * w)
            u2 = H.upsample_fwd(a, n, h, w, 2 * h, 2 * w)
        torch.cuda.synchronize()
        if ref is None:
            ref = (a.clone(), u1.clone())
            continue
        bad[0] += not torch.equal(a, ref[0])
        bad[1] += not torch.equal(u1, ref[1])
        bad[2] += not torch.equal(u2, ref[1])
        for uu in (u1, u2):
            if not torch.equal(uu, ref[1]):
                idx = (uu != ref[1]).nonzero()[:6]
                for r_, c_ in idx.tolist():
                    e, g_ = float(ref[1][r_, c_]), float(uu[r_, c_])
                    print(f"  [{r_},{c_}] want {e:.6g} got {g_:.6g} want*wg {e * float(wg[c_]):.6g} "
                          f"got==ref elsewhere in row: {bool((ref[1][r_] == g_).any())} "
                          f"anywhere: {bool((ref[1] == g_).any())}", flush=True)
        if not torch.equal(u1, ref[1]):
            d = (u1 != ref[1])
            print(f"rep {k}: u1 {int(d.sum())} elems differ, rows {d.any(1).nonzero().flatten()[:8].tolist()}",
                  flush=True)
        del a, u1, u2
    print(f"rank {rank} mode {mode}: a differs {bad[0]}, u1 {bad[1]}, u2 {bad[2]} of {reps - 1}", flush=True)


if __name__ == "__main__":
    main()
