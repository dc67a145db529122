"""Thin torch-tensor wrappers over the C ABI (include/srpde.h).

Activations are 2-D ``[P, C]`` fp32 tensor *views* of NHWC memory (P = N*H*W): a view's
``data_ptr()`` and ``stride(0)`` are exactly the (pointer, ld) pair the kernels take,
so channel slices of a wider buffer (virtual concat, gradient slices) cost nothing.
No function here computes anything on the host; all math runs in libsrpde_hip.so.
"""
from __future__ import annotations

import os

import torch

from ._lib import call, query, stream_ptr

F32 = torch.float32


def _pl(t):
    """(pointer, ld) of a 2-D row-major view."""
    assert t.dim() == 2 and (t.stride(1) == 1 or t.shape[1] == 1), "expected a [P, C] row-major view"
    assert t.dtype == F32 and t.is_cuda, "expected a CUDA fp32 tensor"
    return t.data_ptr(), t.stride(0)


def _p(t):
    return 0 if t is None else t.data_ptr()


def empty(*shape, device):
    return torch.empty(*shape, dtype=F32, device=device)


# ---------------------------------- convolution ------------------------------------
_CONV_MATH = "h3"   # set_conv_math("f32"): the fp32-MFMA kernels (tests, diagnostics)


def set_conv_math(mode: str):
    """Pick the conv kernel family (both HIP, both fp32-accurate):
    'h3': three fp16-split MFMA products with power-of-two operand scales, halo-staged tiles;
    'f32': the fp32 MFMA kernels (also the fallback for shapes h3 does not take)."""
    global _CONV_MATH
    if mode not in ("h3", "f32"):
        raise ValueError(mode)
    _CONV_MATH = mode


# per-kernel accounting (bench.py's roofline): while LAUNCH_TAP is a list, every conv entry call appends
# (kernel name as rocprofv3 prints it -- srpde_last_kernel --, algorithmic FLOP, start event, end event), the
# events recorded on the stream the call launches on
LAUNCH_TAP = None


def _conv_call(name, flop, *args):
    tap = LAUNCH_TAP
    if tap is None:
        return call(name, *args)
    st = torch.cuda.current_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(st)
    call(name, *args)
    b.record(st)
    tap.append((query("srpde_last_kernel").decode(), float(flop), a, b))


def conv_math() -> str:
    return _CONV_MATH


def split_weights_h3(wpack, rows):
    """fp32 packed weights [rows][K] -> ([2, rows*K] fp16 hi/lo planes, [rows] int32 scale
    exponents) for the h3 kernels."""
    K = wpack.numel() // rows
    planes = torch.empty(2, wpack.numel(), dtype=torch.float16, device=wpack.device)
    wexp = torch.empty(rows, dtype=torch.int32, device=wpack.device)
    call("srpde_split_weights_h3", wpack.data_ptr(), planes.data_ptr(), wexp.data_ptr(), rows, K, stream_ptr())
    return planes, wexp


def prepare_weights_h3(desc, nlayers, total_rows):
    """Batched h3 weight split of every conv layer (see unet_exec.prepare_h3_weights)."""
    call("srpde_prepare_weights_h3", desc.data_ptr(), nlayers, total_rows, stream_ptr())


def pack_conv_weights(w, cin_pad, want_fwd=True, want_dgrad=False):
    """Packed fp32 weights (fwd [Cout][tap][Cin], dgrad [Cin][tap][Cout]); in h3 mode each
    packed tensor carries its fp16 split planes and row scales as ``.h3``."""
    cout, cin_real, kh, _ = w.shape
    taps = kh * kh
    wf = empty(cout * taps * cin_pad, device=w.device) if want_fwd else None
    wd = empty(cout * taps * cin_pad, device=w.device) if want_dgrad else None
    call("srpde_pack_conv_weights", w.data_ptr(), _p(wf), _p(wd), cout, cin_pad, cin_real, kh, stream_ptr())
    if _CONV_MATH == "h3" and kh == 3:
        if wf is not None and cin_pad % 32 == 0 and cout % 16 == 0:
            wf.h3 = split_weights_h3(wf, cout)
        if wd is not None and cin_pad % 16 == 0 and cout % 32 == 0:
            wd.h3 = split_weights_h3(wd, cin_pad)
        elif wd is not None and cin_pad % 16 == 0 and cout % 16 == 0:
            # out_conv2 (16 channels): the h3 dgrad reads dy as 32-channel planes (bn_bwd_apply_split pads
            # them), so its split is of the [Cin][tap][32] packing with zero weights for the padded
            # channels; the fp32 packing stays [Cin][tap][16] for the fp32 kernels on a 16-channel dy
            wpad = torch.zeros(cpad32(cout), cin_real, kh, kh, device=w.device)
            wpad[:cout] = w
            wdp = empty(wpad.shape[0] * taps * cin_pad, device=w.device)
            call("srpde_pack_conv_weights", wpad.data_ptr(), 0, wdp.data_ptr(), wpad.shape[0], cin_pad, cin_real, kh,
                 stream_ptr())
            wd.h3 = split_weights_h3(wdp, cin_pad)
    return wf, wd


def cpad32(c):
    """c rounded up to the 32-channel h3 chunk: the channel count of a dy split (bn_bwd_apply_split)."""
    return -(-c // 32) * 32


def conv_stats_buffer(n, h, w, cout, device, c0, c1=0, dil=1):
    """BN-statistics partials for the forward conv of input channels (c0, c1) -> cout: the
    kernel family that will run decides the row-block size.  -> (buffer, blocks, rows/block)."""
    h3 = h3_capable(c0, c1, cout, w, dil)
    rows = (int(query("srpde_conv_h3_stats_rows_for", c0, c1, cout, h, w, dil, _FAMILY)) if h3
            else int(query("srpde_conv_stats_rows_per_block", cout)))
    nblk = -(-(n * h * w) // rows)
    buf = empty(nblk, cout, 2, device=device)
    buf._srpde_rows = rows
    return buf, nblk, rows


# kernel-family bits (include/srpde.h SRPDE_FAM_*): srpde_conv_fwd_h3 / _presplit take them in their accumulate
# argument, srpde_conv_h3_stats_rows_for in its flags -- per call, the library keeps no state.  _FAMILY is the
# bits this module passes (0: the fastest kernels); set_h3r / set_h4 / set_h5 switch a family off for the tests
# that compare the bit-identical families and for tuning.
FAM_NO_H5, FAM_NO_H4, FAM_NO_H3R = 2, 4, 8
_FAMILY = 0


def _set_family(bit, on):
    global _FAMILY
    prev = not (_FAMILY & bit)
    _FAMILY = (_FAMILY & ~bit) if on else (_FAMILY | bit)
    return prev


def set_h3r(on: bool) -> bool:
    """h3 kernel choice for output tiles of <= 64 channels: the register-staged 4-wave kernel
    (two workgroups per CU) or the 8-wave one.  Returns the previous choice."""
    return _set_family(FAM_NO_H3R, bool(on))


def set_h4(on: bool) -> bool:
    """Kernel choice for 128-column h3 tiles at W = 10 / 20: the h4 kernel (conv_h4.hip) or the h3
    8-wave one (bit-identical).  Returns the previous choice."""
    return _set_family(FAM_NO_H4, bool(on))


def set_h5(on: bool) -> bool:
    """Kernel choice for the W = 40 forward into 64 / 32 channels: the h5 kernel (conv_h5.hip) or h4 / h3
    (equal conv outputs; 80- vs 128-row statistics blocks).  Returns the previous choice."""
    return _set_family(FAM_NO_H5, bool(on))


def h3_capable(c0, c1, cout, w, dil, ksize=3):
    return _CONV_MATH == "h3" and bool(query("srpde_conv_h3_supported", c0, c1, cout, w, dil, ksize))


class UpsampledInput:
    """up(x): the bilinear x2 (align_corners) upsample of the NHWC rows ``x`` ([n h w, c]) -- models.py:70,
    89, 92 -- that is not formed: the decoder conv reading it as x0 interpolates its operand tile from x's
    low-res rows (srpde_conv_fwd_h3 x0_up).  ``materialize()`` forms it (srpde_upsample_bilinear_fwd)."""
    __slots__ = ("x", "n", "h", "w", "_t")

    def __init__(self, x, n, h, w):
        self.x, self.n, self.h, self.w, self._t = x, n, h, w, None

    @property
    def shape(self):
        return (self.n * 4 * self.h * self.w, self.x.shape[1])

    @property
    def device(self):
        return self.x.device

    @property
    def is_cuda(self):
        return self.x.is_cuda

    @property
    def _srpde_amax(self):   # a bound on |up(x)|: interpolation is a convex combination
        return amax_of(self.x)

    def materialize(self):
        if self._t is None:
            self._t = tag_amax(upsample_fwd(self.x, self.n, self.h, self.w, 2 * self.h, 2 * self.w),
                               getattr(self.x, "_srpde_amax", None))
        return self._t


def conv_fwd_up_capable(c0, c1, cout, w, dil):
    """Whether conv_fwd takes an UpsampledInput x0 for this shape (the h4 instantiations)."""
    return (_CONV_MATH == "h3" and dil == 1 and ((w == 20 and cout % 128 == 0) or (w == 40 and cout % 64 == 0))
            and bool(query("srpde_conv_h3_supported", c0, c1, cout, w, dil, 3))
            and not (_FAMILY & FAM_NO_H4))


def upsample_gate_sa(x, n, h, w, ho, wo, wg, bg):
    """The spatial attention of the gate whose gating input is up(x), from x alone (srpde_upsample_gate_sa)."""
    sa = empty(n * ho * wo, device=x.device)
    ws = _scratch(int(query("srpde_upsample_gate_sa_workspace_size", n, h, w)), x.device)
    px, ldx = _pl(x)
    call("srpde_upsample_gate_sa", px, ldx, n, h, w, ho, wo, x.shape[1], wg.data_ptr(), bg.data_ptr(), sa.data_ptr(),
         ws.data_ptr(), ws.numel(), stream_ptr())
    return sa


def conv_fwd(x0, x1, wpack, bias, y, n, h, w, cout, ksize=3, dil=1, sign=1, accumulate=False, stats=None,
             planes_out=None, in_affine=None, bn_bwd=None, out_max=None, ep_bn=None, x1_gate=None):
    """Convolution (sign +1) or its input gradient (sign -1, dgrad-packed weights).  h3 only:
    ``planes_out`` ([2, P, c0+c1] fp16) receives the scaled split of the input for conv_wgrad;
    ``in_affine = (scale, shift)`` applies relu(x0 * scale + shift) to the input on the fly;
    ``bn_bwd = (bn_y, mean, invstd, gamma, beta, part)`` (dgrad into a BN + ReLU output's
    gradient) also writes that BN backward's reduction into ``part`` (bn_bwd_partials);
    ``ep_bn = (mean, invstd, gamma, beta, amax)`` (eval mode) applies the following BatchNorm and
    ReLU in the epilogue, so ``y`` is the activation, and writes max|y| into ``amax``.
    ``x1_gate = (ca [n, c1], sa [P])``: x1 is an AttentionGate's input and the conv reads its gated
    output (x1 * ca) * sa, formed in the operand transform (the gated tensor is never written).
    ``x0`` may be an UpsampledInput (h4 shapes, forward): its operand is interpolated from x0.x's rows."""
    up = x0 if isinstance(x0, UpsampledInput) else None
    c1_ = x1.shape[1] if x1 is not None else 0
    if up is not None and not (_CONV_MATH == "h3" and sign == 1 and in_affine is None
                               and conv_fwd_up_capable(x0.shape[1], c1_, cout, w, dil)
                               # statistics: the upsampled-input kernel writes h3 row blocks, so a shape whose
                               # statistics blocks are h5's reads the formed tensor
                               and (stats is None or int(query("srpde_conv_h3_stats_rows_for", x0.shape[1], c1_,
                                                                 cout, h, w, dil, _FAMILY))
                                    == int(query("srpde_conv_h3_stats_rows")))):
        x0 = up.materialize()
        up = None
    p0, ld0 = _pl(x0.x if up is not None else x0)
    if x1 is not None:
        p1, ld1 = _pl(x1)
        c1 = x1.shape[1]
    else:
        p1, ld1, c1 = 0, 0, 0
    py, ldy = _pl(y)
    ws = _scratch(int(query("srpde_conv_fwd_workspace_size", cout)), y.device)
    if _CONV_MATH == "h3" and query("srpde_conv_h3_supported", x0.shape[1], c1, cout, w, dil, ksize):
        planes, wexp = getattr(wpack, "h3", None) or split_weights_h3(wpack, cout)
        rows_fwd = (int(query("srpde_conv_h3_stats_rows_for", x0.shape[1], c1, cout, h, w, dil, _FAMILY)) if sign == 1
                    else int(query("srpde_conv_h3_stats_rows")))
        for buf, rows in ((stats, rows_fwd), (bn_bwd[5] if bn_bwd is not None else None,
                                              int(query("srpde_conv_h3_stats_rows")))):
            if buf is not None and getattr(buf, "_srpde_rows", None) != rows:
                raise ValueError("statistics buffer not laid out for the h3 kernel (use conv_stats_buffer "
                                 "with the input channels / bn_bwd_partials)")
        a0 = amax_of(x0)
        a1 = amax_of(x1) if x1 is not None else None
        _conv_call("srpde_conv_fwd_h3", 2.0 * cout * (x0.shape[1] + c1) * ksize * ksize * n * h * w, p0, x0.shape[1], ld0, p1, c1, ld1, a0.data_ptr(), _p(a1), planes.data_ptr(),
             wexp.data_ptr(), _p(bias), py, ldy, n, h, w, cout, ksize, dil, sign, int(accumulate) | _FAMILY, _p(stats),
             _p(planes_out), _p(in_affine[0] if in_affine else None), _p(in_affine[1] if in_affine else None),
             *_bn_bwd_args(bn_bwd), _p(out_max), *_ep_args(ep_bn), _p(x1_gate[0] if x1_gate else None),
             _p(x1_gate[1] if x1_gate else None), p0 if up is not None else 0, ld0 if up is not None else 0,
             up.h if up is not None else 0, up.w if up is not None else 0, ws.data_ptr(), ws.numel(), stream_ptr())
        if ep_bn is not None:
            tag_amax(y, ep_bn[4])
        if planes_out is not None:
            planes_out._srpde_amax = a0 if a1 is None else (a0, a1)
            planes_out._srpde_c0 = x0.shape[1]
        return
    assert (planes_out is None and in_affine is None and bn_bwd is None and out_max is None
            and x1_gate is None), "planes_out / in_affine / bn_bwd / out_max / x1_gate need the h3 kernels"
    if stats is not None and getattr(stats, "_srpde_rows", None) != int(query("srpde_conv_stats_rows_per_block", cout)):
        raise ValueError("statistics buffer not laid out for this conv family (use conv_stats_buffer)")
    _conv_call("srpde_conv_fwd", 2.0 * cout * (x0.shape[1] + c1) * ksize * ksize * n * h * w, p0, x0.shape[1], ld0, p1, c1, ld1, wpack.data_ptr(), _p(bias), py, ldy,
         n, h, w, cout, ksize, dil, sign, int(accumulate), _p(stats), *_ep_args(ep_bn), ws.data_ptr(), ws.numel(),
         stream_ptr())
    if ep_bn is not None:
        tag_amax(y, ep_bn[4])


def conv_fwd_presplit(xp, wpack, bias, y, n, h, w, cout, ksize=3, dil=1, sign=1, accumulate=False, stats=None,
                      bn_bwd=None, out_max=None):
    """conv_fwd on an input given as its h3 split ``xp`` ([2, P, c] fp16 carrying its max|.| word as
    ``_srpde_amax``: bn_bwd_apply_split's dy, or a stored planes_out) -- srpde_conv_fwd_h3_presplit."""
    c = xp.shape[2]
    planes, wexp = wpack.h3
    py, ldy = _pl(y)
    for buf in (stats, bn_bwd[5] if bn_bwd is not None else None):
        if buf is not None and getattr(buf, "_srpde_rows", None) != int(query("srpde_conv_h3_stats_rows")):
            raise ValueError("statistics buffer not laid out for the h3 kernel")
    ws = _scratch(int(query("srpde_conv_fwd_workspace_size", cout)), y.device)
    _conv_call("srpde_conv_fwd_h3_presplit", 2.0 * cout * c * ksize * ksize * n * h * w, xp.data_ptr(), c, xp._srpde_amax.data_ptr(), planes.data_ptr(), wexp.data_ptr(),
         _p(bias), py, ldy, n, h, w, cout, ksize, dil, sign, int(accumulate) | _FAMILY, _p(stats), *_bn_bwd_args(bn_bwd),
         _p(out_max), ws.data_ptr(), ws.numel(), stream_ptr())


def bn_bwd_apply_split(y, da, mean, invstd, gamma, beta, m1, m2, dy_amax, out=None, relu=True):
    """The BN (+ReLU) backward apply (bn_bwd_prepare's m1 / m2) written as the h3 split of dy:
    [2, P, C] fp16 planes scaled by 2^h3_exp(dy_amax), tagged with that word (srpde_bn_bwd_apply_split)."""
    P, C = y.shape
    py, ldy = _pl(y)
    pda, ldda = _pl(da)
    if out is None:
        out = split_planes_buffer(P, cpad32(C), y.device)
    call("srpde_bn_bwd_apply_split", py, ldy, pda, ldda, mean.data_ptr(), invstd.data_ptr(), gamma.data_ptr(),
         beta.data_ptr(), m1.data_ptr(), m2.data_ptr(), P, C, BN_RELU if relu else 0, dy_amax.data_ptr(),
         out.data_ptr(), stream_ptr())
    out._srpde_amax = dy_amax
    return out


def _ep_args(ep_bn):
    if ep_bn is None:
        return (0, 0, 0, 0, 0)
    mean, invstd, gamma, beta, amax = ep_bn
    return (mean.data_ptr(), invstd.data_ptr(), gamma.data_ptr(), beta.data_ptr(), _p(amax))


_IDENT = {}


def identity_bn(c, device):
    """(mean 0, invstd 1, gamma 1, beta 0) for c channels: the fused BN kernels' pass-through of an
    already activated input (relu((y - 0) * 1 * 1 + 0) == y for y >= 0, exactly)."""
    key = (str(device), c)
    t = _IDENT.get(key)
    if t is None:
        z, o = torch.zeros(c, dtype=F32, device=device), torch.ones(c, dtype=F32, device=device)
        t = _IDENT[key] = (z, o, o, z)
    return t


def _bn_bwd_args(bn_bwd):
    if bn_bwd is None:
        return (0, 0, 0, 0, 0, 0, 0)
    by, mean, invstd, gamma, beta, part = bn_bwd
    pby, ldby = _pl(by)
    return (pby, ldby, mean.data_ptr(), invstd.data_ptr(), gamma.data_ptr(), beta.data_ptr(), part.data_ptr())


def bnb_capable(cout_dy, cin_dx, w, dil):
    """The fused BN-backward dgrad (srpde_conv_dgrad_h3_bnb) covers this layer."""
    return _CONV_MATH == "h3" and bool(query("srpde_conv_h3_bnb_supported", cout_dy, cin_dx, w, dil))


def bn_bwd_prepare(y, da, mean, invstd, gamma, beta, dgamma, dbeta, dbias, relu=True, eval_mode=False, part=None,
                   da_max=None):
    """srpde_bn_bwd_prepare -> (m1, m2, dy_amax word): the BN backward's per-channel terms for
    conv_dgrad_bnb, and its parameter gradients.  ``part`` / ``da_max``: the partials and max|da|
    slots of the dgrad that produced ``da`` (else a reduction pass over y and da)."""
    P, C = y.shape
    py, ldy = _pl(y)
    pda, ldda = _pl(da)
    m1, m2 = empty(C, device=y.device), empty(C, device=y.device)
    # the bound word is written whole by the coefficient kernel: no zero fill (a kernel launch per BN backward)
    word = torch.empty(1, dtype=torch.int32, device=y.device)
    ws_bytes = int(query("srpde_bn_bwd_prepare_workspace_size", P, C))
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=y.device)
    if part is not None and da_max is None:
        da_max = amax_of(da).view(torch.float32)     # max|da| as a one-slot float array
    flags = (BN_RELU if relu else 0) | (BN_EVAL if eval_mode else 0)
    call("srpde_bn_bwd_prepare", py, ldy, pda, ldda, mean.data_ptr(), invstd.data_ptr(), gamma.data_ptr(),
         beta.data_ptr(), P, C, flags, _p(part), part.shape[0] if part is not None else 0, _p(da_max),
         da_max.numel() if (part is not None) else 0, m1.data_ptr(), m2.data_ptr(), _p(dgamma), _p(dbeta), _p(dbias),
         word.data_ptr(), ws.data_ptr(), ws_bytes, stream_ptr())
    return m1, m2, word


def dx_max_slots(n, h, w, cin_dx, device):
    """Per-tile max|dx| slots written by conv_dgrad_bnb (256-row tiles x 64/32-column tiles)."""
    bn = 64 if cin_dx % 64 == 0 else 32
    return empty(-(-(n * h * w) // 256) * -(-cin_dx // bn), device=device)


def out_max_slots(n, h, w, cin, cout, dil, device):
    """Per-tile max|y| slots written by conv_fwd(out_max=...) (srpde_conv_h3_tiles: its tile choice)."""
    t = query("srpde_conv_h3_tiles", n * h * w, cin, cout, w, dil)
    assert t > 0, "out_max_slots: shape not on the h3 kernels"
    return empty(t, device=device)


def conv_dgrad_bnb(da, y, mean, invstd, gamma, beta, m1, m2, dy_amax, wpack, dx, n, h, w, cout_dy, cin_dx, dil,
                   dysplit, relu=True, bn_bwd=None, dx_max=None):
    """srpde_conv_dgrad_h3_bnb: dx = conv^T(dy) with the BN (+ReLU) backward applied on the fly
    (dy = gamma*invstd*(dz - m1 - xhat*m2) from da and y); dy's split goes to ``dysplit``."""
    planes, wexp = wpack.h3
    pda, ldda = _pl(da)
    py, ldy = _pl(y)
    pdx, lddx = _pl(dx)
    for buf in (bn_bwd[5] if bn_bwd is not None else None,):
        if buf is not None and getattr(buf, "_srpde_rows", None) != int(query("srpde_conv_h3_stats_rows")):
            raise ValueError("statistics buffer not laid out for the h3 kernel (bn_bwd_partials)")
    ws = _scratch(int(query("srpde_conv_fwd_workspace_size", cin_dx)), dx.device)
    _conv_call("srpde_conv_dgrad_h3_bnb", 2.0 * cin_dx * cout_dy * 9 * n * h * w, pda, ldda, dy_amax.data_ptr(), py, ldy, mean.data_ptr(), invstd.data_ptr(),
         gamma.data_ptr(), beta.data_ptr(), m1.data_ptr(), m2.data_ptr(), BN_RELU if relu else 0, planes.data_ptr(),
         wexp.data_ptr(), pdx, lddx, n, h, w, cout_dy, cin_dx, dil, dysplit.data_ptr(), *_bn_bwd_args(bn_bwd),
         _p(dx_max), ws.data_ptr(), ws.numel(), stream_ptr())
    dysplit._srpde_amax = dy_amax


def bn_bwd_partials(n, h, w, c, device):
    """Buffer for conv_fwd(bn_bwd=...) (an h3 dgrad): [blocks, c, 2] fp32, h3 row blocks."""
    rows = int(query("srpde_conv_h3_stats_rows"))
    buf = empty(-(-(n * h * w) // rows), c, 2, device=device)
    buf._srpde_rows = rows
    return buf


# ---------------------- operand-scale words of the h3 convolutions ----------------------
# A tensor that feeds an h3 convolution carries ``._srpde_amax``: a 1-element int32 device
# tensor holding max|x| as float bits (an upper bound suffices).  Producers fill it on the
# fly (bn_relu_fwd / bn_relu_bwd); ops whose output is bounded by their input (max-pool,
# bilinear upsample, attention gating) pass the input's word on (tag_amax).
class AmaxSlots:
    """A zeroed block of max|x| words, handed out one per produced activation."""

    def __init__(self, n, device):
        self.buf = torch.zeros(n, dtype=torch.int32, device=device)
        self.next = 0
        self.eval_epilogue = False   # unet_forward: inference forward, BN + ReLU in the conv epilogues

    def take(self):
        if self.next >= self.buf.numel():
            raise RuntimeError("AmaxSlots exhausted")
        self.next += 1
        return self.buf[self.next - 1:self.next]


def tag_amax(t, slot):
    if slot is not None:
        t._srpde_amax = slot
    return t


def amax_of(x):
    """The max|x| word of ``x``: its tag, else computed now (one HIP reduction)."""
    a = getattr(x, "_srpde_amax", None)
    if a is None:
        a = torch.zeros(1, dtype=torch.int32, device=x.device)
        px, ld = _pl(x)
        call("srpde_absmax", px, ld, x.shape[1], x.shape[0], a.data_ptr(), stream_ptr())
    return a


_SCRATCH = {}


def _scratch(nbytes, device):
    """Per-device scratch reused by stream-ordered kernels (tail-split partial tiles)."""
    key = (device.type, device.index)
    buf = _SCRATCH.get(key)
    if buf is None or buf.numel() < nbytes:
        buf = torch.empty(nbytes, dtype=torch.uint8, device=device)
        _SCRATCH[key] = buf
    return buf


def conv_wgrad_bnb(da, y, mean, invstd, gamma, beta, m1, m2, x0, dw, n, h, w, ksize=3, dil=1, relu=True):
    """srpde_conv_wgrad_bnb: the fp32 weight gradient whose dY is the layer's BN (+ReLU) backward (m1 / m2 of
    bn_bwd_prepare) applied as it is loaded -- dy is never written."""
    cout = da.shape[1]
    pda, ldda = _pl(da)
    py, ldy = _pl(y)
    p0, ld0 = _pl(x0)
    cin = x0.shape[1]
    cin_real = dw.shape[1]
    ws_bytes = int(query("srpde_conv_wgrad_workspace_size", n, h, w, cout, cin, ksize))
    ws = torch.empty(max(ws_bytes, 16), dtype=torch.uint8, device=da.device)
    _conv_call("srpde_conv_wgrad_bnb", 2.0 * cout * cin_real * ksize * ksize * n * h * w, pda, ldda, py, ldy,
               mean.data_ptr(), invstd.data_ptr(), gamma.data_ptr(), beta.data_ptr(), m1.data_ptr(), m2.data_ptr(),
               BN_RELU if relu else 0, p0, cin, ld0, dw.data_ptr(), cin_real, 0, n, h, w, cout, ksize, dil,
               ws.data_ptr(), ws_bytes, stream_ptr())


def conv_wgrad(dy, x0, x1, dw, n, h, w, ksize=3, dil=1, accumulate=False):
    cout = dy.shape[1]
    pdy, lddy = _pl(dy)
    p0, ld0 = _pl(x0)
    if x1 is not None:
        p1, ld1 = _pl(x1)
        c1 = x1.shape[1]
    else:
        p1, ld1, c1 = 0, 0, 0
    cin = x0.shape[1] + c1
    cin_real = dw.shape[1]
    ws_bytes = int(query("srpde_conv_wgrad_workspace_size", n, h, w, cout, cin, ksize))
    ws = torch.empty(max(ws_bytes, 16), dtype=torch.uint8, device=dy.device)
    if _CONV_MATH == "h3" and x0.shape[1] % 32 == 0 and c1 % 32 == 0 and cout % 16 == 0 and ksize == 3:
        a1 = amax_of(x1) if x1 is not None else None
        _conv_call("srpde_conv_wgrad_h3", 2.0 * cout * cin_real * ksize * ksize * n * h * w, pdy, lddy, amax_of(dy).data_ptr(), p0, x0.shape[1], ld0, amax_of(x0).data_ptr(),
             p1, c1, ld1, _p(a1), dw.data_ptr(), cin_real, int(accumulate), n, h, w, cout, ksize, dil, ws.data_ptr(),
             ws_bytes, stream_ptr())
        return
    _conv_call("srpde_conv_wgrad", 2.0 * cout * cin_real * ksize * ksize * n * h * w, pdy, lddy, p0, x0.shape[1], ld0, p1, c1, ld1, dw.data_ptr(), cin_real,
         int(accumulate), n, h, w, cout, ksize, dil, ws.data_ptr(), ws_bytes, stream_ptr())


def split_planes_buffer(P, c, device):
    """[2, P, c] fp16 buffer for the h3 kernels' stored input split (planes_out)."""
    return torch.empty(2, P, c, dtype=torch.float16, device=device)


class XSource:
    """The input of a forward whose split the weight gradient forms itself (srpde_conv_wgrad_h3x) instead
    of reading stored planes: what that forward read -- x0, x1, its fused input BN (``in_affine``), the
    attention gate of x1 (``x1_gate``) -- and its max|.| words.  Stands where the stored split ``xp``
    would (conv_wgrad_h3p takes either)."""

    def __init__(self, x0, x1, in_affine, x1_gate):
        self.x0, self.x1, self.in_affine, self.x1_gate = x0, x1, in_affine, x1_gate
        self.a0 = amax_of(x0)
        self.a1 = amax_of(x1) if x1 is not None else None
        for t, a in ((x0, self.a0), (x1, self.a1)):   # the forward then reads the same words
            if t is not None and getattr(t, "_srpde_amax", None) is None:
                t._srpde_amax = a

    def tensors(self):
        """everything the launch reads (kept alive on the weight-gradient stream)"""
        out = [self.x0, self.x1, self.a0, self.a1]
        for t in (self.in_affine or ()) + (self.x1_gate or ()):
            out.append(t)
        return [t for t in out if t is not None]


def wgrad_x_capable(c0, c1, cout, w, dil):
    """srpde_conv_wgrad_h3x takes this layer (the 40 x 40 layers' h3h weight gradient)"""
    return bool(query("srpde_conv_wgrad_h3x_supported", c0, c1, cout, w, dil))


def conv_wgrad_h3p(dyp, xp, dw, n, h, w, ksize=3, dil=1, accumulate=False):
    """Weight gradient from the stored splits: ``dyp`` from the dgrad conv_fwd(planes_out=...) or
    bn_bwd_apply_split (its channels padded to 32: out_conv2's 16), ``xp`` from the forward
    conv_fwd(planes_out=...), each carrying its max|.| word(s); ``dw`` [Cout, Cin, k, k].
    ``xp`` may be an XSource: the kernel splits the fp32 input rows itself (srpde_conv_wgrad_h3x)."""
    if isinstance(xp, XSource):
        return _conv_wgrad_h3x(dyp, xp, dw, n, h, w, ksize, dil, accumulate)
    cout, cin = dw.shape[0], xp.shape[2]
    assert dyp.shape[2] == cpad32(cout), "dy planes must hold cout rounded up to 32 channels"
    ax = xp._srpde_amax
    a0, a1 = (ax, None) if not isinstance(ax, tuple) else ax
    c1 = 0 if a1 is None else cin - xp._srpde_c0
    c0 = cin - c1
    ws_bytes = int(query("srpde_conv_wgrad_h3p_workspace_size", n, h, w, cout, cin, ksize))
    ws = torch.empty(max(ws_bytes, 16), dtype=torch.uint8, device=dyp.device)
    _conv_call("srpde_conv_wgrad_h3p", 2.0 * cout * dw.shape[1] * ksize * ksize * n * h * w, dyp.data_ptr(), dyp._srpde_amax.data_ptr(), xp.data_ptr(), c0, a0.data_ptr(), c1,
         _p(a1), dw.data_ptr(), dw.shape[1], int(accumulate), n, h, w, cout, ksize, dil, ws.data_ptr(), ws_bytes,
         stream_ptr())


def _conv_wgrad_h3x(dyp, xs, dw, n, h, w, ksize, dil, accumulate):
    cout = dw.shape[0]
    assert dyp.shape[2] == cpad32(cout), "dy planes must hold cout rounded up to 32 channels"
    x0, x1 = xs.x0, xs.x1
    c0, c1 = x0.shape[1], (x1.shape[1] if x1 is not None else 0)
    p0, ld0 = _pl(x0)
    p1, ld1 = _pl(x1) if x1 is not None else (0, 0)
    aff, gate = xs.in_affine, xs.x1_gate
    ws_bytes = int(query("srpde_conv_wgrad_h3p_workspace_size", n, h, w, cout, c0 + c1, ksize))
    ws = torch.empty(max(ws_bytes, 16), dtype=torch.uint8, device=dyp.device)
    _conv_call("srpde_conv_wgrad_h3x", 2.0 * cout * dw.shape[1] * ksize * ksize * n * h * w, dyp.data_ptr(),
               dyp._srpde_amax.data_ptr(), p0, ld0, c0, xs.a0.data_ptr(), _p(aff[0] if aff else None),
               _p(aff[1] if aff else None), p1, ld1, c1, _p(xs.a1), _p(gate[0] if gate else None),
               _p(gate[1] if gate else None), dw.data_ptr(), dw.shape[1], int(accumulate), n, h, w, cout, ksize, dil,
               ws.data_ptr(), ws_bytes, stream_ptr())


# ---------------------------------- batch norm -------------------------------------
# the two-pass finalize (srpde_bn_train_finalize_ws; _FIN_SPLIT False: the one-block-per-channel kernel) from
# this many partials per channel: the 40 x 40 layers' 20,480 (36 -> 12 us); at 800-3,200 (20 x 20, 10 x 10) the
# one-pass kernel's 8.5-11.7 us is no slower than the two launches' ~12 (profiles/r05f_bn_finalize_ab.txt)
_FIN_SPLIT = True
_FIN_SPLIT_MIN_BLOCKS = 8192


def _fin_ws(nblk, C, device):
    n = int(query("srpde_bn_finalize_workspace_size", nblk, C))
    return torch.empty(max(n, 16), dtype=torch.uint8, device=device), n


def bn_train_finalize(stats, nblk, rows_per_blk, P, running_mean, running_var, nbt, momentum, eps):
    C = stats.shape[1]
    mean = empty(C, device=stats.device)
    invstd = empty(C, device=stats.device)
    if _FIN_SPLIT and nblk >= _FIN_SPLIT_MIN_BLOCKS:
        ws, n = _fin_ws(nblk, C, stats.device)
        call("srpde_bn_train_finalize_ws", stats.data_ptr(), nblk, rows_per_blk, P, C, _p(running_mean),
             _p(running_var), _p(nbt), float(momentum), float(eps), mean.data_ptr(), invstd.data_ptr(), 0, 0, 0, 0, 0,
             ws.data_ptr(), n, stream_ptr())
        return mean, invstd
    call("srpde_bn_train_finalize", stats.data_ptr(), nblk, rows_per_blk, P, C, _p(running_mean),
         _p(running_var), _p(nbt), float(momentum), float(eps), mean.data_ptr(), invstd.data_ptr(), stream_ptr())
    return mean, invstd


def bn_train_finalize_affine(stats, nblk, rows_per_blk, P, running_mean, running_var, nbt, momentum, eps, gamma,
                             beta, amax=None):
    """bn_train_finalize + bn_affine in one launch -> (mean, invstd, (scale, shift))."""
    C = stats.shape[1]
    dev = stats.device
    mean, invstd, scale, shift = (empty(C, device=dev) for _ in range(4))
    if _FIN_SPLIT and nblk >= _FIN_SPLIT_MIN_BLOCKS:
        ws, n = _fin_ws(nblk, C, dev)
        call("srpde_bn_train_finalize_ws", stats.data_ptr(), nblk, rows_per_blk, P, C, _p(running_mean),
             _p(running_var), _p(nbt), float(momentum), float(eps), mean.data_ptr(), invstd.data_ptr(),
             gamma.data_ptr(), beta.data_ptr(), scale.data_ptr(), shift.data_ptr(), _p(amax), ws.data_ptr(), n,
             stream_ptr())
        return mean, invstd, (scale, shift)
    call("srpde_bn_train_finalize_affine", stats.data_ptr(), nblk, rows_per_blk, P, C, _p(running_mean),
         _p(running_var), _p(nbt), float(momentum), float(eps), mean.data_ptr(), invstd.data_ptr(), gamma.data_ptr(),
         beta.data_ptr(), scale.data_ptr(), shift.data_ptr(), _p(amax), stream_ptr())
    return mean, invstd, (scale, shift)


def bn_affine(mean, invstd, gamma, beta, P, amax=None):
    """(scale, shift) with relu(y * scale + shift) == the train-mode BN + ReLU output, and a
    rigorous max|output| bound written into ``amax`` (the fused consumer's operand scale)."""
    C = mean.numel()
    scale, shift = empty(C, device=mean.device), empty(C, device=mean.device)
    call("srpde_bn_affine", mean.data_ptr(), invstd.data_ptr(), gamma.data_ptr(), beta.data_ptr(), C, P,
         scale.data_ptr(), shift.data_ptr(), _p(amax), stream_ptr())
    return scale, shift


def bn_eval_prepare(running_mean, running_var, eps):
    C = running_mean.numel()
    mean = empty(C, device=running_mean.device)
    invstd = empty(C, device=running_mean.device)
    call("srpde_bn_eval_prepare", running_mean.data_ptr(), running_var.data_ptr(), C, float(eps),
         mean.data_ptr(), invstd.data_ptr(), stream_ptr())
    return mean, invstd


def bn_relu_fwd(y, mean, invstd, gamma, beta, out, relu=True, amax=None):
    py, ldy = _pl(y)
    po, ldo = _pl(out)
    call("srpde_bn_relu_fwd", py, ldy, mean.data_ptr(), invstd.data_ptr(), gamma.data_ptr(), beta.data_ptr(),
         po, ldo, y.shape[0], y.shape[1], int(relu), _p(amax), stream_ptr())
    tag_amax(out, amax)


def bn_relu_pool_fwd(y, mean, invstd, gamma, beta, out, pool, n, h, w, relu=True, amax=None):
    """bn_relu_fwd into ``out`` and maxpool_fwd of it into ``pool`` in one pass."""
    py, ldy = _pl(y)
    po, ldo = _pl(out)
    pp, ldp = _pl(pool)
    call("srpde_bn_relu_pool_fwd", py, ldy, mean.data_ptr(), invstd.data_ptr(), gamma.data_ptr(), beta.data_ptr(),
         po, ldo, pp, ldp, n, h, w, y.shape[1], int(relu), _p(amax), stream_ptr())
    tag_amax(out, amax)
    tag_amax(pool, amax)


def bn_relu_pool_att_fwd(y, mean, invstd, gamma, beta, out, pool, n, h, w, att_params, amax=None):
    """bn_relu_pool_fwd that also returns the attention gate's channel branch (m, hb, ca) of ``out``;
    ``att_params`` = (w1, b1, w2, b2) of its two 1x1 convs."""
    C = y.shape[1]
    dev = y.device
    m, hb, ca = empty(n, C, device=dev), empty(n, C // 8, device=dev), empty(n, C, device=dev)
    py, ldy = _pl(y)
    po, ldo = _pl(out) if out is not None else (0, 0)
    pp, ldp = _pl(pool) if pool is not None else (0, 0)
    w1, b1, w2, b2 = att_params
    call("srpde_bn_relu_pool_att_fwd", py, ldy, mean.data_ptr(), invstd.data_ptr(), gamma.data_ptr(),
         beta.data_ptr(), po, ldo, pp, ldp, n, h, w, C, _p(amax), w1.data_ptr(), b1.data_ptr(), w2.data_ptr(),
         b2.data_ptr(), m.data_ptr(), hb.data_ptr(), ca.data_ptr(), stream_ptr())
    if out is not None:
        tag_amax(out, amax)
    if pool is not None:
        tag_amax(pool, amax)
    return m, hb, ca


def bn_relu_gate_fwd(y, mean, invstd, gamma, beta, out, wg, bg, amax=None):
    """bn_relu_fwd into ``out`` that also returns sa = sigmoid(conv1x1(out; wg, bg)) [P]."""
    P, C = y.shape
    sa = empty(P, device=y.device)
    py, ldy = _pl(y)
    po, ldo = _pl(out) if out is not None else (0, 0)
    call("srpde_bn_relu_gate_fwd", py, ldy, mean.data_ptr(), invstd.data_ptr(), gamma.data_ptr(), beta.data_ptr(),
         po, ldo, P, C, wg.data_ptr(), bg.data_ptr(), sa.data_ptr(), _p(amax), stream_ptr())
    if out is not None:
        tag_amax(out, amax)
    return sa


BN_RELU, BN_EVAL = 1, 2   # srpde_bn_relu_bwd flags (include/srpde.h)


def bn_relu_bwd(y, da, mean, invstd, gamma, beta, dy, dgamma, dbeta, dbias, relu=True, amax=None, part=None,
                eval_mode=False):
    """BN (+ReLU) backward; ``part`` = the reduction already produced by conv_fwd(bn_bwd=...).
    ``eval_mode``: the forward used the running statistics (no batch-statistic terms)."""
    P, C = y.shape
    py, ldy = _pl(y)
    pda, ldda = _pl(da)
    pdy, lddy = _pl(dy)
    ws_bytes = int(query("srpde_bn_relu_bwd_workspace_size", P, C))
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=y.device)
    args = (py, ldy, pda, ldda, mean.data_ptr(), invstd.data_ptr(), gamma.data_ptr(), beta.data_ptr(), pdy, lddy,
            _p(dgamma), _p(dbeta), _p(dbias), P, C, (BN_RELU if relu else 0) | (BN_EVAL if eval_mode else 0), _p(amax))
    if part is None:
        call("srpde_bn_relu_bwd", *args, ws.data_ptr(), ws_bytes, stream_ptr())
    else:
        call("srpde_bn_relu_bwd_part", *args, part.data_ptr(), part.shape[0], ws.data_ptr(), ws_bytes, stream_ptr())
    tag_amax(dy, amax)


# ------------------------------ pool / upsample / misc -----------------------------
def nchw_to_nhwc(x, cpad):
    n, c, h, w = x.shape
    out = empty(n * h * w, cpad, device=x.device)
    call("srpde_nchw_to_nhwc", x.data_ptr(), out.data_ptr(), n, c, h, w, cpad, stream_ptr())
    return out


def nhwc_to_nchw(x, n, c, h, w):
    """[P, >=c] rows -> contiguous [n, c, h, w] (srpde_nhwc_to_nchw)."""
    px, ldx = _pl(x)
    out = torch.empty(n, c, h, w, dtype=F32, device=x.device)
    call("srpde_nhwc_to_nchw", px, ldx, out.data_ptr(), n, c, h, w, stream_ptr())
    return out


def axpy_(y, x, channel=0, channels=1, alpha=1.0):
    """y[:, channel] += alpha * x for y [n, channels, h, w] and x [n * h * w] (srpde_axpy_channel)."""
    n = y.shape[0]
    hw = y[0, 0].numel()
    call("srpde_axpy_channel", y.data_ptr(), x.data_ptr(), n, channels, hw, channel, float(alpha), stream_ptr())


def maxpool_fwd(x, n, h, w):
    c = x.shape[1]
    out = empty(n * (h // 2) * (w // 2), c, device=x.device)
    px, ldx = _pl(x)
    call("srpde_maxpool2x2_fwd", px, ldx, out.data_ptr(), c, n, h, w, c, stream_ptr())
    return tag_amax(out, getattr(x, "_srpde_amax", None))


def maxpool_bwd(x, dout, dx, n, h, w, accumulate):
    px, ldx = _pl(x)
    pdo, lddo = _pl(dout)
    pdx, lddx = _pl(dx)
    call("srpde_maxpool2x2_bwd", px, ldx, pdo, lddo, pdx, lddx, n, h, w, x.shape[1], int(accumulate), stream_ptr())


def upsample_fwd(x, n, h, w, ho, wo, out=None):
    c = x.shape[1]
    if out is None:
        out = empty(n * ho * wo, c, device=x.device)
    px, ldx = _pl(x)
    po, ldo = _pl(out)
    call("srpde_upsample_bilinear_fwd", px, ldx, po, ldo, n, h, w, ho, wo, c, stream_ptr())
    return tag_amax(out, getattr(x, "_srpde_amax", None))   # convex combinations of inputs


def upsample_gate_fwd(x, n, h, w, ho, wo, wg, bg):
    """upsample_fwd plus the spatial attention of the gate that reads it -> (out, sa)."""
    c = x.shape[1]
    out = empty(n * ho * wo, c, device=x.device)
    sa = empty(n * ho * wo, device=x.device)
    px, ldx = _pl(x)
    po, ldo = _pl(out)
    call("srpde_upsample_bilinear_gate_fwd", px, ldx, po, ldo, n, h, w, ho, wo, c, wg.data_ptr(), bg.data_ptr(),
         sa.data_ptr(), stream_ptr())
    return tag_amax(out, getattr(x, "_srpde_amax", None)), sa


def att_apply_fwd(x, n, hw, chan, sa, out=None):
    """The gate's output from att_channel_fwd's ``chan`` and a precomputed spatial attention ``sa``.
    Returns (out, saved) as att_fwd."""
    m, hb, ca = chan
    c = x.shape[1]
    if out is None:
        out = empty(n * hw, c, device=x.device)
    px, ldx = _pl(x)
    po, ldo = _pl(out)
    call("srpde_att_apply_fwd", px, ldx, n, hw, c, ca.data_ptr(), sa.data_ptr(), po, ldo, stream_ptr())
    tag_amax(out, getattr(x, "_srpde_amax", None))
    return out, (m, hb, ca, sa)


def resize_bicubic(x, ho, wo):
    """F.interpolate(mode='bicubic', align_corners=True) of single-channel fields: x [planes, h, w]
    contiguous fp32 -> [planes, ho, wo] (srpde_resize_bicubic_ac)."""
    if not (x.is_cuda and x.dtype == F32 and x.is_contiguous() and x.dim() == 3):
        raise RuntimeError("resize_bicubic: contiguous fp32 [planes, h, w] ROCm tensor (no CPU fallback)")
    pl, h, w = x.shape
    out = torch.empty(pl, ho, wo, dtype=F32, device=x.device)
    call("srpde_resize_bicubic_ac", x.data_ptr(), out.data_ptr(), pl, h, w, ho, wo, stream_ptr())
    return out


def pde_dataset_assemble(u_coarse, u_fine, theta_fine, f_fine, stats, theta_constant):
    """srpde_pde_dataset_assemble: -> (inputs [N, 3, hf, wf], targets [N, 1, hf, wf])."""
    n, hc, wc = u_coarse.shape
    _, hf, wf = u_fine.shape
    for t in (u_coarse, u_fine, theta_fine, f_fine, stats):
        if not (t.is_cuda and t.dtype == F32 and t.is_contiguous()):
            raise RuntimeError("pde_dataset_assemble: contiguous fp32 ROCm tensors only (no CPU fallback)")
    if theta_fine.shape != u_fine.shape or f_fine.shape != u_fine.shape or stats.numel() != 6:
        raise ValueError("pde_dataset_assemble: theta / f must match u_fine's shape, stats has 6 entries")
    inputs = torch.empty(n, 3, hf, wf, dtype=F32, device=u_fine.device)
    targets = torch.empty(n, 1, hf, wf, dtype=F32, device=u_fine.device)
    call("srpde_pde_dataset_assemble", u_coarse.data_ptr(), u_fine.data_ptr(), theta_fine.data_ptr(),
         f_fine.data_ptr(), stats.data_ptr(), int(theta_constant), n, hc, wc, hf, wf, inputs.data_ptr(),
         targets.data_ptr(), stream_ptr())
    return inputs, targets


def upsample_bwd(dout, dx, n, h, w, ho, wo, accumulate, gate=None, bn=None):
    """``gate = (dsa, wg)``: the upsampled tensor's gradient is dout + dsa (x) wg (the attention
    gating gradient left unapplied by att_bwd(dg=None)).  ``bn = (y, mean, invstd, gamma, beta)``: the BN +
    ReLU whose output gradient dx is; returns its backward reduction (part [n*h, c, 2], da_max [n*h]) formed
    from the stored values (srpde_upsample_bilinear_bwd_gated_bn), or None when the shape has no fused
    kernel (the BN backward then reduces on its own)."""
    pdo, lddo = _pl(dout)
    pdx, lddx = _pl(dx)
    if bn is not None and gate is not None and not accumulate and bool(
            query("srpde_upsample_bwd_bn_supported", h, w, ho, wo, dx.shape[1], lddo, lddx)):
        y, mean, invstd, gamma, beta = bn
        dsa, wg = gate
        py, ldy = _pl(y)
        c = dx.shape[1]
        part = empty(n * h, c, 2, device=dx.device)
        da_max = empty(n * h, device=dx.device)
        call("srpde_upsample_bilinear_bwd_gated_bn", pdo, lddo, dsa.data_ptr(), wg.data_ptr(), pdx, lddx, n, h, w, ho,
             wo, c, py, ldy, mean.data_ptr(), invstd.data_ptr(), gamma.data_ptr(), beta.data_ptr(), BN_RELU,
             part.data_ptr(), da_max.data_ptr(), stream_ptr())
        return part, da_max
    if gate is not None:
        dsa, wg = gate
        call("srpde_upsample_bilinear_bwd_gated", pdo, lddo, dsa.data_ptr(), wg.data_ptr(), pdx, lddx, n, h, w, ho,
             wo, dx.shape[1], int(accumulate), stream_ptr())
        return None
    call("srpde_upsample_bilinear_bwd", pdo, lddo, pdx, lddx, n, h, w, ho, wo, dx.shape[1], int(accumulate),
         stream_ptr())
    return None


def gating_bn_reduce(dsa, wg, dg, y, mean, invstd, gamma, beta):
    """dg += dsa (x) wg (the gating gradient att_bwd(dg=None) left out) with the backward reduction of the BN +
    ReLU whose output gradient dg is -> (part [blocks, C, 2], da_max [blocks]) (srpde_gating_bn_reduce)."""
    P, C = y.shape
    pdg, lddg = _pl(dg)
    py, ldy = _pl(y)
    nb = int(query("srpde_gating_bn_reduce_blocks", P, C))
    part = empty(nb, C, 2, device=dg.device)
    da_max = empty(nb, device=dg.device)
    call("srpde_gating_bn_reduce", dsa.data_ptr(), wg.data_ptr(), pdg, lddg, py, ldy, mean.data_ptr(),
         invstd.data_ptr(), gamma.data_ptr(), beta.data_ptr(), P, C, BN_RELU, part.data_ptr(), da_max.data_ptr(),
         stream_ptr())
    return part, da_max


# ----------------------------------- attention -------------------------------------
def att_fwd(x, g, n, hw, w1, b1, w2, b2, wg, bg, out=None):
    c, gc = x.shape[1], g.shape[1]
    dev = x.device
    m = empty(n, c, device=dev)
    hb = empty(n, c // 8, device=dev)
    ca = empty(n, c, device=dev)
    sa = empty(n * hw, device=dev)
    if out is None:
        out = empty(n * hw, c, device=dev)
    px, ldx = _pl(x)
    pg, ldg = _pl(g)
    po, ldo = _pl(out)
    call("srpde_att_fwd", px, ldx, pg, ldg, n, hw, c, gc, w1.data_ptr(), b1.data_ptr(), w2.data_ptr(),
         b2.data_ptr(), wg.data_ptr(), bg.data_ptr(), m.data_ptr(), hb.data_ptr(), ca.data_ptr(), sa.data_ptr(),
         po, ldo, stream_ptr())
    tag_amax(out, getattr(x, "_srpde_amax", None))   # x * sigmoid * sigmoid: |out| <= |x|
    return out, (m, hb, ca, sa)


def att_channel_fwd(x, n, hw, w1, b1, w2, b2):
    """srpde_att_channel_fwd -> (m, hb, ca): the gate's channel attention (x alone)."""
    c = x.shape[1]
    dev = x.device
    m, hb, ca = empty(n, c, device=dev), empty(n, c // 8, device=dev), empty(n, c, device=dev)
    px, ldx = _pl(x)
    call("srpde_att_channel_fwd", px, ldx, n, hw, c, w1.data_ptr(), b1.data_ptr(), w2.data_ptr(), b2.data_ptr(),
         m.data_ptr(), hb.data_ptr(), ca.data_ptr(), stream_ptr())
    return m, hb, ca


def att_gate_fwd(x, g, n, hw, chan, wg, bg, out=None):
    """srpde_att_gate_fwd with ``chan`` = att_channel_fwd(x, ...): out = x * ca * sigmoid(conv1x1(g)).
    Returns (out, saved) as att_fwd."""
    m, hb, ca = chan
    c, gc = x.shape[1], g.shape[1]
    sa = empty(n * hw, device=x.device)
    if out is None:
        out = empty(n * hw, c, device=x.device)
    px, ldx = _pl(x)
    pg, ldg = _pl(g)
    po, ldo = _pl(out)
    call("srpde_att_gate_fwd", px, ldx, pg, ldg, n, hw, c, gc, ca.data_ptr(), wg.data_ptr(), bg.data_ptr(),
         sa.data_ptr(), po, ldo, stream_ptr())
    tag_amax(out, getattr(x, "_srpde_amax", None))   # x * sigmoid * sigmoid: |out| <= |x|
    return out, (m, hb, ca, sa)


def att_bwd(dout, x, g, n, hw, w1, w2, wg, saved, dx, dx_acc, dg, dg_acc, dw1, db1, dw2, db2, dwg, dbg,
            defer_params=False, want_dsa=False, want_dm=False, g_lowres=None):
    """AttentionGate backward.  Returns (dsa or None, params): ``dsa`` (when ``dg`` is None, or
    ``want_dsa``) is the gating gradient's per-pixel factor d loss / d(spatial pre-activation), for
    upsample_bwd(gate=...); the spatial bias gradient is its sum; ``params`` (when
    ``defer_params``) is a callable that launches the parameter-gradient reductions on the
    current stream, to be queued after this call (reads ``ws``, ``g``, ``m``, ``hb``).
    ``dx=None``: the input gradient is left to att_pool_bn_bwd; ``want_dm`` then appends the channel
    branch's term dm [n, c] (a view into the workspace) to the returned tuple.  ``g_lowres = (d, h, w, ho, wo)``:
    g is up(d), and the spatial conv's weight gradient is formed from the low-res d
    (srpde_att_bwd_params_lowres)."""
    m, hb, ca, sa = saved
    c, gc = x.shape[1], g.shape[1]
    ws_bytes = int(query("srpde_att_bwd_workspace_size", n, hw, c, gc))
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=x.device)
    pdo, lddo = _pl(dout)
    px, ldx = _pl(x)
    pg, ldg = _pl(g)
    pdx, lddx = _pl(dx) if dx is not None else (0, 0)
    pdg, lddg = _pl(dg) if dg is not None else (0, 0)
    pgrads = (dw1.data_ptr(), db1.data_ptr(), dw2.data_ptr(), db2.data_ptr(), dwg.data_ptr(), dbg.data_ptr())
    later = defer_params or g_lowres is not None   # the parameter pass as its own call (below)
    call("srpde_att_bwd", pdo, lddo, px, ldx, pg, ldg, n, hw, c, gc, w1.data_ptr(), w2.data_ptr(), wg.data_ptr(),
         m.data_ptr(), hb.data_ptr(), ca.data_ptr(), sa.data_ptr(), pdx, lddx, int(dx_acc), pdg, lddg, int(dg_acc),
         *((0,) * 6 if later else pgrads), ws.data_ptr(), ws_bytes, stream_ptr())
    params = None
    if later:
        if g_lowres is not None:
            d, h, w, ho, wo = g_lowres
            pd, ldd = _pl(d)

            def params():
                call("srpde_att_bwd_params_lowres", pd, ldd, n, h, w, ho, wo, c, gc, m.data_ptr(), hb.data_ptr(),
                     *pgrads, ws.data_ptr(), ws_bytes, stream_ptr())
            params.keep = (ws, d)
        else:
            def params():
                call("srpde_att_bwd_params", pg, ldg, n, hw, c, gc, m.data_ptr(), hb.data_ptr(), *pgrads,
                     ws.data_ptr(), ws_bytes, stream_ptr())
            params.keep = (ws,)
        if not defer_params:   # in line: the same parameter pass, now
            params()
            params = None
    # the gating gradient's per-pixel factor, for upsample_bwd(gate=(dsa, wg))
    dsa = ws[:4 * x.shape[0]].view(torch.float32) if dg is None or want_dsa else None
    if want_dm:   # workspace [P floats of dsa | n * c floats of dm | ...] (srpde_att_bwd_workspace_size)
        P = x.shape[0]
        return dsa, params, ws[4 * P:4 * (P + n * c)].view(torch.float32).view(n, c)
    return dsa, params


def att_pool_bn_bwd(dout, ca, sa, dm, a, dp, de, y, mean, invstd, gamma, beta, n, h, w):
    """srpde_att_pool_bn_bwd: de = the AttentionGate's input gradient ((dout * sa) * ca + dm, att_bwd's with
    dx=None) + the max-pool backward of dp over a, written once, and the BatchNorm (y, mean, invstd, gamma,
    beta; + ReLU) backward's partial sums of de -> (part [blocks, c, 2], da_max [blocks]) for
    bn_bwd_prepare(part=..., da_max=...)."""
    c = a.shape[1]
    nb = int(query("srpde_att_pool_bn_bwd_blocks", n, h, w, c))
    part = empty(nb, c, 2, device=a.device)
    da_max = empty(nb, device=a.device)
    pdo, lddo = _pl(dout)
    pa, lda = _pl(a)
    pdp, lddp = _pl(dp)
    py, ldy = _pl(y)
    pde, ldde = _pl(de)
    call("srpde_att_pool_bn_bwd", pdo, lddo, ca.data_ptr(), sa.data_ptr(), dm.data_ptr(), pa, lda, pdp, lddp, py, ldy,
         mean.data_ptr(), invstd.data_ptr(), gamma.data_ptr(), beta.data_ptr(), pde, ldde, n, h, w, c,
         part.data_ptr(), da_max.data_ptr(), stream_ptr())
    return part, da_max


# ------------------------------------- head ----------------------------------------
def conv_head_eval(z, wpack, bias, mean, invstd, gamma, beta, wf, bf, xin, n, h, w):
    """out_conv2 -> BN (eval) -> ReLU -> final -> + residual in one pass (srpde_conv_head_eval) -> [n h w]."""
    planes, wexp = wpack.h3
    out = empty(n * h * w, device=z.device)
    pz, ldz = _pl(z)
    _conv_call("srpde_conv_head_eval", 2.0 * 16 * 32 * 9 * n * h * w, pz, ldz, amax_of(z).data_ptr(), planes.data_ptr(), wexp.data_ptr(), _p(bias),
         mean.data_ptr(), invstd.data_ptr(), gamma.data_ptr(), beta.data_ptr(), wf.data_ptr(), bf.data_ptr(),
         xin.data_ptr(), xin.shape[1], n, h, w, out.data_ptr(), stream_ptr())
    return out


def head_fwd(z, wf, bf, xin, n, hw):
    out = empty(n * hw, device=z.device)
    pz, ldz = _pl(z)
    call("srpde_head_fwd", pz, ldz, z.shape[1], wf.data_ptr(), bf.data_ptr(), xin.data_ptr(), xin.shape[1],
         n, hw, out.data_ptr(), stream_ptr())
    return out


def head_bwd(dout, z, wf, n, hw, dz, dwf, dbf):
    pz, ldz = _pl(z)
    pdz, lddz = _pl(dz)
    c = z.shape[1]
    ws_bytes = int(query("srpde_head_bwd_workspace_size", n, hw, c))
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=z.device)
    call("srpde_head_bwd", dout.data_ptr(), pz, ldz, c, wf.data_ptr(), n, hw, pdz, lddz, dwf.data_ptr(),
         dbf.data_ptr(), ws.data_ptr(), ws_bytes, stream_ptr())


# -------------------------------------- MSE ----------------------------------------
def mse_fwd(y, t):
    ws_bytes = int(query("srpde_mse_workspace_size"))
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=y.device)
    loss = torch.empty((), dtype=F32, device=y.device)
    call("srpde_mse_fwd", y.data_ptr(), t.data_ptr(), y.numel(), loss.data_ptr(), ws.data_ptr(), ws_bytes,
         stream_ptr())
    return loss


def mse_bwd(y, t, gout):
    dy = torch.empty_like(y)
    call("srpde_mse_bwd", y.data_ptr(), t.data_ptr(), y.numel(), _p(gout), dy.data_ptr(), stream_ptr())
    return dy


# ----------------------------------- optimizer -------------------------------------
def clip_coef(flat_grad, grad_scale, max_norm, coef):
    ws_bytes = int(query("srpde_grad_norm_workspace_size"))
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=flat_grad.device)
    call("srpde_clip_coef", flat_grad.data_ptr(), flat_grad.numel(), float(grad_scale), float(max_norm),
         coef.data_ptr(), ws.data_ptr(), ws_bytes, stream_ptr())


def adamw_step(p, g, m, v, lr, beta1, beta2, eps, wd, step, coef, grad_scale):
    call("srpde_adamw_step", p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), p.numel(), float(lr),
         float(beta1), float(beta2), float(eps), float(wd), int(step), _p(coef), float(grad_scale), stream_ptr())
