"""Whole-network HIP executor for the attention U-Net (forward + backward).

Restates reference ``UNet.forward`` (src/models.py:72-101) as an explicit schedule of
libsrpde_hip.so launches over NHWC ``[P, C]`` buffers, and its autograd backward as the
reverse schedule.  Design points:

* torch.cat never materialises: the decoder convs read ``(x0, x1)`` as a virtual
  concat, and their dgrad writes one ``[P, C0+C1]`` gradient whose two slices are the
  gradients of the two concat inputs (the attention-gating gradient accumulates into
  the first slice in place).
* ``up(d3)`` / ``up(d2)`` are computed once (the reference computes each twice,
  models.py:89-93; the values are identical).
* BatchNorm batch statistics come from the conv epilogue; the backward recomputes x_hat
  and the ReLU mask from the saved conv output.
* Parameter gradients are written straight into one flat buffer laid out in
  *backward-completion order*, so a data-parallel reducer can all-reduce finished
  prefixes while the rest of the backward still runs (``grad_ready`` hook).
"""
from __future__ import annotations

import contextlib

import torch

from . import hipops as H

# forward-pass module groups; the flat parameter buffer uses the REVERSE of this order
FORWARD_GROUPS = ["enc1", "enc2", "enc3", "bridge", "att3", "dec3", "att2", "dec2", "att1", "dec1",
                  "out_conv1", "out_bn1", "out_conv2", "out_bn2", "final"]
FLAT_GROUPS = list(reversed(FORWARD_GROUPS))


def flat_layout(model):
    """[(name, param, offset, numel)] in flat (backward-completion) order."""
    named = dict(model.named_parameters())
    out, off = [], 0
    for grp in FLAT_GROUPS:
        for name, p in named.items():
            if name == grp or name.startswith(grp + "."):
                out.append((name, p, off, p.numel()))
                off += p.numel()
    assert off == sum(p.numel() for p in named.values()), "flat layout does not cover every parameter"
    return out


def _group_end_offsets(layout):
    ends = {}
    for name, _, off, n in layout:
        grp = next(g for g in FLAT_GROUPS if name == g or name.startswith(g + "."))
        ends[grp] = max(ends.get(grp, 0), off + n)
    return ends


class _Saved:
    pass


# diagnostics hook (tools/diag_stages.py): when a dict, unet_backward stores a copy of each
# named activation gradient as soon as it is final
DEBUG_TAPS = None


def _tap(name, t):
    if DEBUG_TAPS is not None:
        DEBUG_TAPS[name] = t.detach().clone()


def _tap_dgrad(conv, dyp, dx, dx_max, out_part):
    if DEBUG_TAPS is not None:
        name = getattr(conv, "_srpde_name", "?")
        for k, t in (("dyp", dyp), ("dx", dx), ("dx_max", dx_max), ("bn_part", out_part)):
            if t is not None:
                _tap(f"{k}:{name}", t)


# bench/profiling hook: {conv module name: list} -> (start, end) HIP events recorded on the
# compute stream around that layer's forward conv launch
TIMED_LAYERS = {}


def _conv_launch(conv, *args, **kw):
    sink = TIMED_LAYERS.get(getattr(conv, "_srpde_name", None)) if TIMED_LAYERS else None
    if sink is None:
        H.conv_fwd(*args, **kw)
        return
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    H.conv_fwd(*args, **kw)
    b.record()
    sink.append((a, b, H.query("srpde_last_kernel").decode()))


class GatedInput:
    """An AttentionGate's output (x * ca) * sa (models.py:119-130) that is not formed: the decoder conv
    that reads it as the second half of its virtual concat applies the gate in its operand transform
    (srpde_conv_fwd_h3 x1_ca / x1_sa), so the gated tensor is never written or read back.
    ``materialize()`` forms it (srpde_att_apply_fwd) for a consumer that cannot fuse it."""
    __slots__ = ("x", "ca", "sa", "n", "hw", "_t")

    def __init__(self, x, ca, sa, n, hw):
        self.x, self.ca, self.sa, self.n, self.hw, self._t = x, ca, sa, n, hw, None

    @property
    def shape(self):
        return self.x.shape

    @property
    def device(self):
        return self.x.device

    def materialize(self):
        if self._t is None:
            self._t, _ = H.att_apply_fwd(self.x, self.n, self.hw, (None, None, self.ca), self.sa)
        return self._t


def _unwrap_gate(x0, x1, cout, w, dil):
    """-> (x1 tensor, x1_gate or None) for a conv whose second input may be a GatedInput."""
    if not isinstance(x1, GatedInput):
        return x1, None
    if _FUSE_ATT_APPLY and H.h3_capable(x0.shape[1], x1.shape[1], cout, w, dil):
        return x1.x, (x1.ca, x1.sa)
    return x1.materialize(), None


class _Planes:
    """Holder of one packed weight tensor's h3 split: ``.h3 = (planes, row exponents)``."""
    __slots__ = ("h3",)

    def __init__(self, planes, wexp):
        self.h3 = (planes, wexp)


def prepare_h3_weights(m):
    """Split every 3x3 conv's weights into h3 planes (forward and dgrad packings) with ONE
    launch per step (srpde_prepare_weights_h3), instead of a pack + split per layer and pass.
    Buffers and the layer table persist on the model; they are rebuilt if a weight moves."""
    if H.conv_math() != "h3":
        return
    convs = [mod for mod in m.modules() if isinstance(mod, torch.nn.Conv2d) and mod.kernel_size == (3, 3)]
    sig = tuple(c.weight.data_ptr() for c in convs)
    cache = getattr(m, "_srpde_h3w", None)
    if cache is None or cache[0] != sig:
        dev = convs[0].weight.device
        rows, desc, keep = 0, [], []
        for c in convs:
            cout, cin = c.out_channels, c.in_channels
            pf = ef = pd = ed = None
            if cin % 32 == 0 and cout % 16 == 0:
                pf = torch.empty(2, cout * 9 * cin, dtype=torch.float16, device=dev)
                ef = torch.empty(cout, dtype=torch.int32, device=dev)
            if cout % 16 == 0 and cin % 16 == 0:   # dgrad rows k = tap * cpad32(cout) + n (out_conv2: 16 -> 32)
                pd = torch.empty(2, cin * 9 * H.cpad32(cout), dtype=torch.float16, device=dev)
                ed = torch.empty(cin, dtype=torch.int32, device=dev)
            c._srpde_h3f = _Planes(pf, ef) if pf is not None else None
            c._srpde_h3d = _Planes(pd, ed) if pd is not None else None
            if pf is None and pd is None:
                continue
            # a layer owns cout forward rows then cin dgrad rows (rows of a missing packing idle)
            desc.append([c.weight.data_ptr(), cout, cin, cin, H._p(pf), H._p(ef), H._p(pd), H._p(ed), rows,
                         H.cpad32(cout)])
            rows += cout + cin
            keep += [t for t in (pf, ef, pd, ed) if t is not None]
        cache = (sig, torch.tensor(desc, dtype=torch.int64, device=dev), len(desc), rows, keep)
        m._srpde_h3w = cache
    _, desc_t, nl, rows, _ = cache
    # eval mode: the split stays valid until a weight changes (in place through torch: version
    # counters; through FusedAdamW's kernel: its step count); train mode re-splits every forward
    key = None
    if not m.training:
        from .optim import step_count
        key = (sig, tuple(c.weight._version for c in convs), step_count())
        if getattr(m, "_srpde_h3w_key", None) == key:
            return
    global _H3W_PENDING
    dev = desc_t.device
    if _H3W_SIDE and m.training and dev.type == "cuda" and not torch.cuda.is_current_stream_capturing():
        # on the side stream, beside the input transpose and enc1.conv1 (which reads no split):
        # the first consumer of a split waits for it (_h3w_ready)
        main = torch.cuda.current_stream(dev)
        side = WgradStream(dev).side
        side.wait_stream(main)
        with torch.cuda.stream(side):
            H.prepare_weights_h3(desc_t, nl, rows)
        _H3W_PENDING = torch.cuda.Event()
        _H3W_PENDING.record(side)
    else:
        H.prepare_weights_h3(desc_t, nl, rows)
    m._srpde_h3w_key = key


# the per-step weight split on the side stream (_H3W_SIDE False: in line); its event until the
# first h3 convolution of the step waits for it
_H3W_SIDE = True
_H3W_PENDING = None


# DataParallel's buffer broadcast (distributed.py), issued on a side stream before the forward: the
# compute stream waits for its event before the step's first BatchNorm finalize
_BUF_PENDING = None


def buffers_pending(event):
    global _BUF_PENDING
    _BUF_PENDING = event


def _buffers_ready(dev):
    global _BUF_PENDING
    if _BUF_PENDING is not None:
        torch.cuda.current_stream(dev).wait_event(_BUF_PENDING)
        _BUF_PENDING = None


def _h3w_ready(dev):
    global _H3W_PENDING
    if _H3W_PENDING is not None:
        torch.cuda.current_stream(dev).wait_event(_H3W_PENDING)
        _H3W_PENDING = None


def _fwd_weights(conv, cin, c0, c1, w, dil):
    wp = getattr(conv, "_srpde_h3f", None)
    if wp is not None and H.h3_capable(c0, c1, conv.out_channels, w, dil):
        _h3w_ready(conv.weight.device)
        return wp
    return H.pack_conv_weights(conv.weight, cin)[0]


def _dgrad_weights(conv, cin, w, dil, cdy=None):
    """The dgrad's packed weights for a dy operand of ``cdy`` channels (default: the layer's output
    channels).  The cached h3 planes hold cpad32(cout) dy channels (out_conv2: 16 padded to 32, the
    planes of bn_bwd_apply_split); a 16-channel fp32 dy takes the fp32 packing instead."""
    cdy = conv.out_channels if cdy is None else cdy
    wp = getattr(conv, "_srpde_h3d", None)
    if wp is not None and cdy == H.cpad32(conv.out_channels) and H.h3_capable(cdy, 0, cin, w, dil):
        _h3w_ready(conv.weight.device)
        return wp
    return H.pack_conv_weights(conv.weight, cin, want_fwd=False, want_dgrad=True)[1]


def _splits_both_ways(c0, c1, cout, w, dil):
    """The layer's forward and dgrad both run on h3, so its weight gradient reads stored splits (the
    dgrad reads dy as planes of cpad32(cout) channels: out_conv2's 16 padded to 32, which only the
    pre-split BN backward apply produces)."""
    return (H.h3_capable(c0, c1, cout, w, dil) and H.h3_capable(H.cpad32(cout), 0, c0 + c1, w, dil)
            and (cout % 32 == 0 or _PRESPLIT_BWD))


def _cbr_fwd(conv, bn, x0, x1, n, h, w, training, dil, slots, in_affine=None, activate=True, pool=False, att=None,
             gate=None):
    """conv3x3 -> BatchNorm2d -> ReLU  (ConvBlock half, models.py:22-23; bridge :43-48).

    ``activate=False`` (train mode): stop after the BN statistics and return the conv output y
    with the (scale, shift) that a fused consumer applies (``in_affine``) instead of a
    materialised relu(bn(y)); y carries the rigorous max|relu(bn(y))| bound as its amax word.
    ``pool``: also return the 2x2 max-pool of the activation, formed in the same pass
    (srpde_bn_relu_pool_fwd): ((a, pooled), saved).  With ``att`` (the AttentionGate that reads a)
    also its channel branch, from the same pass when possible (srpde_bn_relu_pool_att_fwd):
    ((a, pooled, early), saved), ``early`` as _att_channel_early returns it.  ``gate``: the
    AttentionGate whose gating input a is; returns ((a, sa), saved) with its spatial attention."""
    dev = x0.device
    cout = conv.out_channels
    c1 = x1.shape[1] if x1 is not None else 0
    cin = x0.shape[1] + c1
    wf = _fwd_weights(conv, cin, x0.shape[1], c1, w, dil)
    x1_saved = x1
    x1, x1_gate = _unwrap_gate(x0, x1, cout, w, dil)
    P = n * h * w
    y = H.empty(P, cout, device=dev)
    xp = None
    if training:
        stats, nblk, rpb = H.conv_stats_buffer(n, h, w, cout, dev, x0.shape[1], c1, dil)
        if _splits_both_ways(x0.shape[1], c1, cout, w, dil):
            if (_WGRAD_X and not isinstance(x0, H.UpsampledInput) and x0.is_cuda
                    and H.wgrad_x_capable(x0.shape[1], c1, cout, w, dil)):
                # the weight gradient splits the fp32 input itself (srpde_conv_wgrad_h3x): nothing stored
                xp = H.XSource(x0, x1, in_affine, x1_gate)
            else:
                xp = H.split_planes_buffer(P, cin, dev)   # the input's split, kept for the weight gradient
        assert in_affine is None or xp is not None, "a fused input needs the stored split for its wgrad"
        _conv_launch(conv, x0, x1, wf, conv.bias, y, n, h, w, cout, 3, dil, 1, False, stats,
                     None if isinstance(xp, H.XSource) else xp, in_affine, x1_gate=x1_gate)
        mom = bn.momentum if bn.momentum is not None else 0.0
        _buffers_ready(dev)
        _RS_EPOCH[0] += 1   # the finalize below rewrites the running statistics torch's version counters miss
        if not activate:   # the fused consumer's (scale, shift), from the same launch (_FIN_AFFINE False: two)
            slot = slots.take()
            if _FIN_AFFINE:
                mean, invstd, aff = H.bn_train_finalize_affine(stats, nblk, rpb, P, bn.running_mean, bn.running_var,
                                                               bn.num_batches_tracked, mom, bn.eps, bn.weight,
                                                               bn.bias, amax=slot)
            else:
                mean, invstd = H.bn_train_finalize(stats, nblk, rpb, P, bn.running_mean, bn.running_var,
                                                   bn.num_batches_tracked, mom, bn.eps)
                aff = H.bn_affine(mean, invstd, bn.weight, bn.bias, P, amax=slot)
            y._srpde_amax = slot
            return (y, aff), (None if in_affine is not None else x0, x1_saved, y, mean, invstd, xp, training)
        mean, invstd = H.bn_train_finalize(stats, nblk, rpb, P, bn.running_mean, bn.running_var,
                                           bn.num_batches_tracked, mom, bn.eps)
    else:
        assert in_affine is None and activate
        mean, invstd = _eval_stats(bn)
        if getattr(slots, "eval_epilogue", False) and _EVAL_EPI and H.h3_capable(x0.shape[1], c1, cout, w, dil):
            # inference: the conv epilogue applies this BN (running statistics) + ReLU, so y IS the
            # activation (nothing saved for a backward); consumers read it as is
            slot = slots.take()
            H.conv_fwd(x0, x1, wf, conv.bias, y, n, h, w, cout, 3, dil, 1, False, None,
                       ep_bn=(mean, invstd, bn.weight, bn.bias, slot), x1_gate=x1_gate)
            return _eval_consumers(y, slot, n, h, w, cout, pool, att, gate), None
        if (getattr(slots, "eval_epilogue", False) and _EVAL_EPI and _EVAL_EPI_F32 and x1 is None and x1_gate is None
                and x0.shape[1] % 32):
            # the same on the register-staged fp32 kernel (enc1.conv1: 3 -> 4 padded input channels)
            slot = slots.take()
            H.conv_fwd(x0, None, wf, conv.bias, y, n, h, w, cout, 3, dil, 1, False, None,
                       ep_bn=(mean, invstd, bn.weight, bn.bias, slot))
            return _eval_consumers(y, slot, n, h, w, cout, pool, att, gate), None
        H.conv_fwd(x0, x1, wf, conv.bias, y, n, h, w, cout, 3, dil, 1, False, None, x1_gate=x1_gate)
    # a fused input is not the layer's real input (that is relu(bn(x0))): keep no reference to it,
    # the weight gradient reads the stored split
    saved = (None if in_affine is not None else x0, x1_saved, y, mean, invstd, xp, training)
    a = H.empty(P, cout, device=dev)
    if gate is not None:
        s0 = gate.spatial_attention[0]
        if _FUSE_SA and cout in (256, 512, 1024):
            return (a, H.bn_relu_gate_fwd(y, mean, invstd, bn.weight, bn.bias, a, s0.weight, s0.bias,
                                          amax=slots.take())), saved
        H.bn_relu_fwd(y, mean, invstd, bn.weight, bn.bias, a, amax=slots.take())
        return (a, None), saved
    if pool and _FUSE_POOL:
        pooled = H.empty(n * (h // 2) * (w // 2), cout, device=dev)
        if att is not None and _per_sample_ok(n, h, w, cout):
            c1, c3, _ = _att_params(att)
            chan = H.bn_relu_pool_att_fwd(y, mean, invstd, bn.weight, bn.bias, a, pooled, n, h, w,
                                          (c1.weight, c1.bias, c3.weight, c3.bias), amax=slots.take())
            return (a, pooled, (chan, None)), saved
        H.bn_relu_pool_fwd(y, mean, invstd, bn.weight, bn.bias, a, pooled, n, h, w, amax=slots.take())
    elif (not pool and att is not None and _per_sample_ok(n, h, w, cout)
          and a.is_cuda and not torch.cuda.is_current_stream_capturing()):
        c1, c3, _ = _att_params(att)
        chan = H.bn_relu_pool_att_fwd(y, mean, invstd, bn.weight, bn.bias, a, None, n, h, w,
                                      (c1.weight, c1.bias, c3.weight, c3.bias), amax=slots.take())
        return (a, (chan, None)), saved
    else:
        H.bn_relu_fwd(y, mean, invstd, bn.weight, bn.bias, a, amax=slots.take())
        if not pool:
            return (a, _att_channel_early(att, a, n, h * w)) if att is not None else a, saved
        pooled = H.maxpool_fwd(a, n, h, w)
    if att is None:
        return (a, pooled), saved
    return (a, pooled, _att_channel_early(att, a, n, h * w)), saved


# the running statistics change in place through torch (version counters: load_state_dict, user
# writes) or through this executor's train-mode BN finalize kernels, which torch cannot see: every
# train-mode forward bumps this epoch
_RS_EPOCH = [0]


def _eval_stats(bn):
    """(mean, 1 / sqrt(var + eps)) of a BatchNorm's running statistics for the eval forward, cached
    until they change (srpde_bn_eval_prepare: one tiny launch per BN layer per forward otherwise)."""
    rm, rv = bn.running_mean, bn.running_var
    if not _EVAL_STATS_CACHE or rm.is_inference() or rv.is_inference():
        # (inference tensors -- buffers of a model built or loaded under torch.inference_mode() -- have no
        # version counter to key a cache on)
        return H.bn_eval_prepare(rm, rv, bn.eps)
    key = (rm.data_ptr(), rm._version, rv.data_ptr(), rv._version, float(bn.eps), _RS_EPOCH[0])
    c = getattr(bn, "_srpde_eval_stats", None)
    if c is None or c[0] != key:
        c = (key, H.bn_eval_prepare(rm, rv, bn.eps))
        bn._srpde_eval_stats = c
    return c[1]


def _eval_consumers(a, slot, n, h, w, c, pool, att, gate):
    """_cbr_fwd's return value for an activation ``a`` the conv epilogue already formed (eval mode):
    the pooled tensor, the gate's channel branch or its spatial attention from the fused passes with
    an identity BN and no activation write."""
    dev = a.device
    ident = H.identity_bn(c, dev)
    if gate is not None:
        s0 = gate.spatial_attention[0]
        if _FUSE_SA and c in (256, 512, 1024):
            return a, H.bn_relu_gate_fwd(a, *ident, None, s0.weight, s0.bias)
        return a, None
    if pool:
        pooled = H.empty(n * (h // 2) * (w // 2), c, device=dev)
        if att is not None and _per_sample_ok(n, h, w, c) and _FUSE_POOL:
            c1, c3, _ = _att_params(att)
            chan = H.bn_relu_pool_att_fwd(a, *ident, None, pooled, n, h, w,
                                          (c1.weight, c1.bias, c3.weight, c3.bias))
            H.tag_amax(pooled, slot)
            return a, pooled, (chan, None)
        pooled = H.maxpool_fwd(a, n, h, w)
        if att is None:
            return a, pooled
        return a, pooled, _att_channel_early(att, a, n, h * w)
    if att is not None:
        if _per_sample_ok(n, h, w, c) and a.is_cuda and not torch.cuda.is_current_stream_capturing():
            c1, c3, _ = _att_params(att)
            chan = H.bn_relu_pool_att_fwd(a, *ident, None, None, n, h, w, (c1.weight, c1.bias, c3.weight, c3.bias))
            return a, (chan, None)
        return a, _att_channel_early(att, a, n, h * w)
    return a


# inference (eval, nothing saved for a backward): BN + ReLU in the conv epilogue (_EVAL_EPI False: the
# separate passes)
_EVAL_EPI = True
# ... also on the register-staged fp32 kernel of enc1.conv1 (_EVAL_EPI_F32 False: its separate BN + ReLU pass)
_EVAL_EPI_F32 = True
# the eval forward's per-layer BN (mean, invstd) cached across forwards (_EVAL_STATS_CACHE False: recomputed)
_EVAL_STATS_CACHE = True
_FUSE_D1 = True
_FIN_AFFINE = True
# the gates' spatial attention formed by the upsample that produces their gating input
# (srpde_upsample_bilinear_gate_fwd; _FUSE_SA False: separate pass over g)
_FUSE_SA = True
# inference: out_conv2 + out_bn2 + ReLU + final + residual in one kernel (srpde_conv_head_eval; _FUSE_HEAD False:
# out_conv2 on the conv kernels, then srpde_head_fwd)
_FUSE_HEAD = True
# inference: the decoder's first convs read up(d) from d's rows (H.UpsampledInput; _FUSE_UP False: formed)
_FUSE_UP = True
# enc1's / enc2's gate channel branch from the BN + ReLU + pool pass (srpde_bn_relu_pool_att_fwd, one
# block per sample; _FUSE_ATT_CH False: a separate pass over the activation)
_FUSE_ATT_CH = True


def _per_sample_ok(n, h, w, c):
    """srpde_bn_relu_pool_att_fwd runs ONE workgroup per sample: take it when the batch fills the
    chip or a sample is small (the 40x40 training / cascade tiles), not for a few large fields
    (e.g. B = 1 at 640^2, where one CU would write the whole activation)."""
    return _FUSE_ATT_CH and c % 32 == 0 and c <= 256 and (n >= 256 or h * w <= 4096)


# a ConvBlock output's BN + ReLU and the max-pool that reads it in one pass (_FUSE_POOL False: two)
_FUSE_POOL = True


class WgradStream:
    """Weight gradients on a second HIP stream.

    Nothing in the backward reads a weight gradient, so the wgrad launches leave the critical
    path (dgrad -> BN backward -> dgrad ...): each is queued on a side stream behind the compute
    stream's work so far, and its MFMA work fills the CUs the dgrad chain leaves idle (tail
    waves, the HBM-bound BN / attention / upsample kernels).  Operands allocated on the compute
    stream are ``record_stream``-ed so the caching allocator does not recycle them early;
    ``join()`` makes the compute stream wait for every queued wgrad (before anything reads the
    gradients)."""

    _streams = {}

    def __init__(self, dev):
        self.main = torch.cuda.current_stream(dev)
        key = (dev.type, dev.index if dev.index is not None else torch.cuda.current_device())
        side = WgradStream._streams.get(key)
        if side is None:
            side = torch.cuda.Stream(device=dev)
            WgradStream._streams[key] = side
        self.side = side

    def submit(self, fn, keep=()):
        self.side.wait_stream(self.main)
        with torch.cuda.stream(self.side):
            fn()
        for t in keep:
            if t is not None:
                t.record_stream(self.side)

    def join(self):
        self.main.wait_stream(self.side)


# weight gradients on a side stream (_WGRAD_STREAM False: in line on the compute stream)
_WGRAD_STREAM = True
# the backward's dgrad chain on a high-priority stream: "1" always, "0" never, unset: only under
# data parallelism.  A high-priority stream never shares a hardware queue with the normal-priority
# weight-gradient stream; with RCCL's streams present the two normal-priority streams were seen
# sharing one queue, which serialised wgrad behind dgrad (DataParallel step 37.9 ms -> 35.7 ms,
# plain step 35.6 ms; without a process group the priority is neutral, 35.74 vs 35.64 ms)
_BWD_PRIORITY = "auto"
_PRIO_STREAMS = {}


def _priority_stream(dev):
    key = (dev.type, dev.index if dev.index is not None else torch.cuda.current_device())
    st = _PRIO_STREAMS.get(key)
    if st is None:
        lo, hi = torch.cuda.Stream.priority_range()   # (lowest, highest): a smaller number is higher
        st = _PRIO_STREAMS[key] = torch.cuda.Stream(device=dev, priority=hi)
    return st


def _xkeep(xp):
    """what an XSource's weight-gradient launch reads (stream-kept like its other operands)"""
    return tuple(xp.tensors()) if isinstance(xp, H.XSource) else ()


def _cbr_bwd(conv, bn, saved, da, n, h, w, dil, grads, slots, dx=None, dx_accumulate=False, part=None,
             below=None, wq=None):
    """dgrad first: its h3 kernel stores dy's split, which the weight gradient then reads together
    with the input's split stored by the forward (h3p); otherwise the splitting wgrad kernels.

    ``part``: this BN's backward reduction, already produced by the dgrad that wrote ``da`` -- a
    (partials, max|da| slots or None) pair.
    ``below = (bn, saved)``: the BN + ReLU whose output this layer reads; when the dgrad runs on
    h3 into a fresh ``dx`` it also produces that BN's reduction, returned for the next call.
    ``wq``: a WgradStream that takes the weight-gradient launch off the compute stream.

    Train mode with an h3 dgrad into ``dx`` of at most 64 channels (one output-column tile) from a
    dy of at least 64 (two 32-channel chunks): the BN (+ReLU) backward is applied inside the
    dgrad's operand transform (srpde_conv_dgrad_h3_bnb), so dy is never written or read in fp32 --
    srpde_bn_bwd_prepare forms the per-channel terms first.  Per layer in the step (same box):
    enc1.conv2 -84 us, dec1.conv2 -44 us, enc2.conv1 ~-120 us; with several output-column tiles
    (dec1.conv1: +108 us, each tile repeats the transform) or a single input chunk (out_conv1:
    +45 us) the separate elementwise pass is cheaper, so those keep it."""
    x0, x1, y, mean, invstd, xp, train = saved
    P, cout = y.shape
    part_t, da_max = part if part is not None else (None, None)
    cin = conv.in_channels if x0 is None else x0.shape[1] + (x1.shape[1] if x1 is not None else 0)
    dyp = None
    out_part = None
    if (_FUSE_BN_APPLY and train and dx is not None and xp is not None and not dx_accumulate
            and cin <= _BNB_MAX_CIN and cout >= _BNB_MIN_COUT and H.bnb_capable(cout, cin, w, dil)):
        m1, m2, dyw = H.bn_bwd_prepare(y, da, mean, invstd, bn.weight, bn.bias, grads[bn.weight], grads[bn.bias],
                                       grads[conv.bias], part=part_t, da_max=da_max)
        wd = _dgrad_weights(conv, cin, w, dil)
        dyp = H.split_planes_buffer(P, cout, y.device)
        bn_bwd, dx_max = None, None
        if below is not None and _FUSE_BN_BWD:
            bnb, sb = below
            out_part = H.bn_bwd_partials(n, h, w, cin, y.device)
            bn_bwd = (sb[2], sb[3], sb[4], bnb.weight, bnb.bias, out_part)
            dx_max = H.dx_max_slots(n, h, w, cin, y.device)
        H.conv_dgrad_bnb(da, y, mean, invstd, bn.weight, bn.bias, m1, m2, dyw, wd, dx, n, h, w, cout, cin, dil, dyp,
                         bn_bwd=bn_bwd, dx_max=dx_max)
        _tap_dgrad(conv, dyp, dx, dx_max, out_part)
        fn, keep = (lambda: H.conv_wgrad_h3p(dyp, xp, grads[conv.weight], n, h, w, 3, dil)), (dyp, dyw) + _xkeep(xp)
        if wq is None:
            fn()
        else:
            wq.submit(fn, keep)
        return None if out_part is None else (out_part, dx_max)
    if (_PRESPLIT_BWD and train and dx is not None and xp is not None
            and H.h3_capable(H.cpad32(cout), 0, cin, w, dil)):
        # the BN backward apply writes dy as its h3 split (scale from bn_bwd_prepare's rigorous bound);
        # the dgrad reads the fp16 pieces straight into its operand tiles and the weight gradient
        # reads the same planes: no fp32 dy, no split work or split store in the dgrad
        m1, m2, dyw = H.bn_bwd_prepare(y, da, mean, invstd, bn.weight, bn.bias, grads[bn.weight], grads[bn.bias],
                                       grads[conv.bias], part=part_t, da_max=da_max)
        dyp = H.bn_bwd_apply_split(y, da, mean, invstd, bn.weight, bn.bias, m1, m2, dyw)
        if DEBUG_TAPS is not None:
            _tap("dyp:" + getattr(conv, "_srpde_name", "?"), dyp)
        wd = _dgrad_weights(conv, cin, w, dil, cdy=H.cpad32(cout))
        bn_bwd, dx_max = None, None
        if below is not None and not dx_accumulate and _FUSE_BN_BWD:
            bnb, sb = below
            out_part = H.bn_bwd_partials(n, h, w, cin, y.device)
            bn_bwd = (sb[2], sb[3], sb[4], bnb.weight, bnb.bias, out_part)
            if _FUSE_BN_APPLY:   # max|dx| slots for the layer below's BN backward bound
                dx_max = H.out_max_slots(n, h, w, H.cpad32(cout), cin, dil, y.device)
        H.conv_fwd_presplit(dyp, wd, None, dx, n, h, w, cin, 3, dil, -1, dx_accumulate, None, bn_bwd=bn_bwd,
                            out_max=dx_max)
        _tap_dgrad(conv, dyp, dx, dx_max, out_part)
        fn, keep = (lambda: H.conv_wgrad_h3p(dyp, xp, grads[conv.weight], n, h, w, 3, dil)), (dyp, dyw) + _xkeep(xp)
        if wq is None:
            fn()
        else:
            wq.submit(fn, keep)
        return None if out_part is None else (out_part, dx_max)
    if (_FUSE_WGRAD_BN and train and dx is None and xp is None and x0 is not None and x1 is None
            and x0.shape[1] % 32 != 0 and DEBUG_TAPS is None):
        # enc1.conv1 (no dgrad: the input image): the fp32 weight gradient applies the BN backward to its dY loads
        m1, m2, _ = H.bn_bwd_prepare(y, da, mean, invstd, bn.weight, bn.bias, grads[bn.weight], grads[bn.bias],
                                     grads[conv.bias], part=part_t, da_max=da_max)
        dw = grads[conv.weight]
        fn = lambda: H.conv_wgrad_bnb(da, y, mean, invstd, bn.weight, bn.bias, m1, m2, x0, dw, n, h, w, 3, dil)
        if wq is None:
            fn()
        else:
            wq.submit(fn, (da, y, m1, m2))
        return None
    dy = H.empty(P, cout, device=y.device)
    # eval mode: the forward normalised with the running statistics (constants), so the BN
    # backward drops the batch-statistic terms (aten native_batch_norm_backward, training=False)
    H.bn_relu_bwd(y, da, mean, invstd, bn.weight, bn.bias, dy, grads[bn.weight], grads[bn.bias], grads[conv.bias],
                  amax=slots.take(), part=part_t, eval_mode=not train)
    if DEBUG_TAPS is not None:
        _tap("dy:" + getattr(conv, "_srpde_name", "?"), dy)
    if dx is not None:
        wd = _dgrad_weights(conv, cin, w, dil)
        if xp is not None:
            dyp = H.split_planes_buffer(P, cout, y.device)
        bn_bwd, dx_max = None, None
        if below is not None and not dx_accumulate and _FUSE_BN_BWD and H.h3_capable(cout, 0, cin, w, dil):
            bnb, sb = below
            out_part = H.bn_bwd_partials(n, h, w, cin, y.device)
            bn_bwd = (sb[2], sb[3], sb[4], bnb.weight, bnb.bias, out_part)
            if _FUSE_BN_APPLY:   # max|dx| slots for a fused BN apply in the layer below
                dx_max = H.out_max_slots(n, h, w, cout, cin, dil, y.device)
        H.conv_fwd(dy, None, wd, None, dx, n, h, w, cin, 3, dil, -1, dx_accumulate, None, dyp, bn_bwd=bn_bwd,
                   out_max=dx_max)
        _tap_dgrad(conv, dyp, dx, dx_max, out_part)
    dw = grads[conv.weight]
    if xp is not None and dyp is not None:
        fn, keep = (lambda: H.conv_wgrad_h3p(dyp, xp, dw, n, h, w, 3, dil)), (dyp, dyp._srpde_amax) + _xkeep(xp)
    else:
        assert x0 is not None, "fused-input layer without stored splits"
        if isinstance(x1, GatedInput):
            x1 = x1.materialize()
        fn, keep = (lambda: H.conv_wgrad(dy, x0, x1, dw, n, h, w, 3, dil)), (dy, getattr(dy, "_srpde_amax", None))
    if wq is None:
        fn()
    else:
        wq.submit(fn, keep)
    return None if out_part is None else (out_part, dx_max)


# the attention gates' output (x * ca) * sa formed inside the decoder conv that reads it (GatedInput;
# _FUSE_ATT_APPLY False: a separate srpde_att_apply_fwd pass writes it)
_FUSE_ATT_APPLY = True

# enc1.conv1's BN backward applied inside its fp32 weight gradient's dY loads (srpde_conv_wgrad_bnb; False: dy
# written by bn_relu_bwd, then read)
_FUSE_WGRAD_BN = True

# the BN (+ReLU) backward apply of a layer fused into its dgrad's operand transform
# (srpde_conv_dgrad_h3_bnb; _FUSE_BN_APPLY False: off)
_FUSE_BN_APPLY = True
# layers it is taken for: dgrad output channels <= _BNB_MAX_CIN (one output-column tile), dy channels
# >= _BNB_MIN_COUT (two input chunks); wider (dec1.conv1's 3-tile dgrad, out_conv1's one-chunk dy)
# measured +0.5 ms in the step
_BNB_MAX_CIN, _BNB_MIN_COUT = 64, 64

# the BN backward apply writes dy as its h3 split for a presplit dgrad (_PRESPLIT_BWD False: fp32 dy,
# split inside the dgrad)
_PRESPLIT_BWD = True

# the 40 x 40 layers' weight gradients split their fp32 input rows themselves (srpde_conv_wgrad_h3x), so
# their training forwards store no input split (_WGRAD_X False: the forward stores it, h3h reads it)
_WGRAD_X = True

# the BN backward reduction of a layer is fused into the dgrad above it (_FUSE_BN_BWD False: off)
_FUSE_BN_BWD = True


def _fuse_pair(conv2, training, w, dil):
    """conv1's BN + ReLU can be applied inside conv2 (never materialised) in train mode when
    conv2 keeps its input split for the weight gradient (so nothing else reads relu(bn(y1)))."""
    return training and _splits_both_ways(conv2.in_channels, 0, conv2.out_channels, w, dil)


def _pair_fwd(conv1, bn1, conv2, bn2, x0, x1, n, h, w, training, dil, slots, pool=False, activate=True, att=None,
              gate=None):
    """conv1 -> BN -> ReLU -> conv2 -> BN -> ReLU, with the middle BN + ReLU fused into conv2's
    input transform when possible (saves a read and a write of the middle activation)."""
    if _fuse_pair(conv2, training, w, dil):
        (y1, aff), s1 = _cbr_fwd(conv1, bn1, x0, x1, n, h, w, training, dil, slots, activate=False)
        a2, s2 = _cbr_fwd(conv2, bn2, y1, None, n, h, w, training, dil, slots, in_affine=aff, pool=pool,
                          activate=activate, att=att, gate=gate)
        return a2, (s1, s2)
    a1, s1 = _cbr_fwd(conv1, bn1, x0, x1, n, h, w, training, dil, slots)
    a2, s2 = _cbr_fwd(conv2, bn2, a1, None, n, h, w, training, dil, slots, pool=pool, activate=activate, att=att,
                      gate=gate)
    return a2, (s1, s2)


def _block_fwd(blk, x0, x1, n, h, w, training, slots, pool=False, activate=True, att=None):
    """``activate=False`` (train mode): the block's output BN + ReLU is left to a fused consumer,
    which gets ((y, (scale, shift)), saved) as from _cbr_fwd(activate=False)."""
    return _pair_fwd(blk.conv1, blk.bn1, blk.conv2, blk.bn2, x0, x1, n, h, w, training, 1, slots, pool=pool,
                     activate=activate, att=att)


# training: up(d3) interpolated inside dec2.conv1's forward (h4 upsampled-input kernel with statistics and the stored
# split) and att2's spatial attention from d3 at low resolution, as in inference: u3 is never written (False: formed)
_TRAIN_UP3 = True
# the decoder gates' spatial weight gradient from the low-res decoder output d (sum_q d[q] up^T(dsa)[q]) instead of
# the upsampled g = up(d), a quarter of the rows (False: from g)
_GATE_WGRAD_LOWRES = True
# bridge[4]'s backward reduction formed with att3's gating gradient (_FUSE_GATING_BN False: the att_bwd dg pass and a
# separate reduction pass)
_FUSE_GATING_BN = True
# the decoder blocks' bn2 backward reduction formed inside the upsample backward (_FUSE_UP_BN False: a
# separate reduction pass re-reads the upsample's output)
_FUSE_UP_BN = True


def _up_bn(blk, saved):
    """(y, mean, invstd, gamma, beta) of ``blk``.bn2 for upsample_bwd(bn=...), or None (_FUSE_UP_BN off)."""
    if not _FUSE_UP_BN:
        return None
    _, _, y, mean, invstd, _, _ = saved[1]
    return y, mean, invstd, blk.bn2.weight, blk.bn2.bias


def _block_bwd(blk, saved, da, n, h, w, grads, slots, dx, dx_accumulate=False, wq=None, part=None, last=False):
    """``part``: bn2's backward reduction, when the dgrad that wrote ``da`` produced it.  ``last``: the backward's
    final block (enc1): conv1's weight gradient runs in line on the compute stream, which would otherwise sit idle
    waiting for the side stream's queue (enc1.conv2's weight gradient) at the join (_INLINE_LAST_WGRAD)."""
    s1, s2 = saved
    P = n * h * w
    da1 = H.empty(P, blk.conv1.out_channels, device=da.device)
    part = _cbr_bwd(blk.conv2, blk.bn2, s2, da, n, h, w, 1, grads, slots, da1, part=part, below=(blk.bn1, s1),
                    wq=wq)
    _cbr_bwd(blk.conv1, blk.bn1, s1, da1, n, h, w, 1, grads, slots, dx, dx_accumulate, part=part,
             wq=None if last and _INLINE_LAST_WGRAD else wq)


# the last block's conv1 weight gradient in line on the compute stream (False: on the side stream, queued behind
# enc1.conv2's, while the compute stream waits at the join)
_INLINE_LAST_WGRAD = True


def _att_params(att):
    c1, c3, s0 = att.channel_attention[1], att.channel_attention[3], att.spatial_attention[0]
    return c1, c3, s0


def _att_fwd(att, x, g, n, hw, early=None, sa=None):
    """``early``: the gate's channel attention already launched by _att_channel_early; ``sa``: its
    spatial attention already formed by the upsample that produced ``g`` (upsample_gate_fwd)."""
    c1, c3, s0 = _att_params(att)
    if early is None:
        return H.att_fwd(x, g, n, hw, c1.weight, c1.bias, c3.weight, c3.bias, s0.weight, s0.bias)
    chan, ev = early
    if ev is not None:
        torch.cuda.current_stream(x.device).wait_event(ev)
    if sa is not None:
        if _FUSE_ATT_APPLY and x.is_cuda:   # formed by the consuming decoder conv (GatedInput)
            m_, hb, ca = chan
            return GatedInput(x, ca, sa, n, hw), (m_, hb, ca, sa)
        return H.att_apply_fwd(x, n, hw, chan, sa)
    return H.att_gate_fwd(x, g, n, hw, chan, s0.weight, s0.bias)


def _upsample_for_gate(d, att, n, h, w, ho, wo, conv=None, c1=0, fuse=False):
    """up(d) for the decoder, and (_FUSE_SA) the spatial attention of ``att`` whose gate it is.
    ``fuse`` (inference; ``conv`` the decoder conv reading up(d) as x0 beside ``c1`` gated channels):
    up(d) is not formed -- an UpsampledInput the conv interpolates from d's rows (_FUSE_UP False: off),
    the gate's spatial attention computed from d at low resolution (srpde_upsample_gate_sa)."""
    if (fuse and _FUSE_UP and _FUSE_SA and _FUSE_ATT_APPLY and d.is_cuda and conv is not None
            and H.conv_fwd_up_capable(d.shape[1], c1, conv.out_channels, wo, 1)):
        s0 = att.spatial_attention[0]
        return H.UpsampledInput(d, n, h, w), H.upsample_gate_sa(d, n, h, w, ho, wo, s0.weight, s0.bias)
    if _FUSE_SA and d.shape[1] in (128, 256) and d.is_cuda:
        s0 = att.spatial_attention[0]
        return H.upsample_gate_fwd(d, n, h, w, ho, wo, s0.weight, s0.bias)
    return H.upsample_fwd(d, n, h, w, ho, wo), None


def _att_channel_early(att, x, n, hw):
    """att's channel attention of x (models.py:119-121: a function of the encoder output alone), in
    line; returns what _att_fwd(early=...) takes."""
    c1, c3, _ = _att_params(att)
    return H.att_channel_fwd(x, n, hw, c1.weight, c1.bias, c3.weight, c3.bias), None


def _att_bwd(att, saved, dout, x, g, n, hw, grads, dx, dx_acc, dg, dg_acc, wq=None, defer_dx=False, g_lowres=None):
    """``dg=None``: the gating gradient is not applied; returns the gate for upsample_bwd.
    ``wq``: the parameter-gradient reductions go to the weight-gradient side stream.
    ``defer_dx`` (``dx`` None): the input gradient is formed later by att_pool_bn_bwd; returns (gate, dm)."""
    c1, c3, s0 = _att_params(att)
    out = H.att_bwd(dout, x, g, n, hw, c1.weight, c3.weight, s0.weight, saved, dx, dx_acc, dg, dg_acc,
                    grads[c1.weight], grads[c1.bias], grads[c3.weight], grads[c3.bias], grads[s0.weight],
                    grads[s0.bias], defer_params=wq is not None, want_dsa=DEBUG_TAPS is not None, want_dm=defer_dx,
                    g_lowres=g_lowres if _GATE_WGRAD_LOWRES else None)
    dsa, params = out[0], out[1]
    if DEBUG_TAPS is not None:
        _tap("dsa_pre:" + getattr(att, "_srpde_name", "?"), dsa)
    if params is not None:
        wq.submit(params, params.keep)
    gate = None if dsa is None or dg is not None else (dsa, s0.weight)
    return (gate, out[2]) if defer_dx else gate


def _fuse_enc_out(blk_saved, c, w):
    """The encoder output's gradient (gate input + max-pool backward) and its BN backward reduction in one pass
    (srpde_att_pool_bn_bwd): train mode, c / 4 a power of two <= 64 (_FUSE_ENC_OUT False: three passes)"""
    s2 = blk_saved[1]
    return _FUSE_ENC_OUT and s2[6] and c in (64, 128, 256) and w % 2 == 0


def _enc_out_bwd(blk, blk_saved, att_saved, dout, dm, e, dp, de, n, h, w):
    """de = the gate's input gradient + the max-pool backward of dp; -> (partials, max|de| slots) of blk.bn2"""
    _, s2 = blk_saved
    _, _, y, mean, invstd, _, _ = s2
    _, _, ca, sa = att_saved
    return H.att_pool_bn_bwd(dout, ca, sa, dm, e, dp, de, y, mean, invstd, blk.bn2.weight, blk.bn2.bias, n, h, w)


# the encoder outputs' gradient in one pass with their BN backward reduction (False: the gate's input gradient,
# the max-pool backward and the reduction as three passes; tests/test_gpu_fused_bwd.py compares the two)
_FUSE_ENC_OUT = True


def check_input(x):
    if x.dim() != 4 or x.shape[1] != 3:
        raise ValueError(f"UNet expects [B, 3, H, W] input, got {tuple(x.shape)}")
    if x.shape[2] % 4 or x.shape[3] % 4:
        raise ValueError("UNet needs H and W divisible by 4 (two 2x2 pools)")
    if not x.is_cuda or x.dtype != torch.float32:
        raise RuntimeError("the HIP U-Net runs on a ROCm device in float32 (no CPU fallback)")


def unet_forward(m, x, training, save=False):
    """UNet.forward (models.py:72-101).  Returns (out [B,1,H,W], saved-or-None)."""
    check_input(x)
    x = x.contiguous()
    n, _, h, w = x.shape
    h2, w2, h3, w3 = h // 2, w // 2, h // 4, w // 4
    hw1, hw2, hw3 = h * w, h2 * w2, h3 * w3
    if training:
        _RS_EPOCH[0] += 1   # this forward's BN finalize kernels rewrite the running statistics
    S = _Saved()
    S.shape = (n, h, w)
    S.x = x
    x4 = H.nchw_to_nhwc(x, 4)
    S.x4 = x4
    prepare_h3_weights(m)
    # max|x| words of the 16 BN+ReLU outputs (h3 operand scales)
    slots = H.AmaxSlots(16, x.device)
    slots.eval_epilogue = not training and not save   # inference: BN + ReLU in the conv epilogues
    # encoder
    (e1, p1, ch1), S.enc1 = _block_fwd(m.enc1, x4, None, n, h, w, training, slots, pool=True, att=m.att1)
    (e2, p2, ch2), S.enc2 = _block_fwd(m.enc2, p1, None, n, h2, w2, training, slots, pool=True, att=m.att2)
    (e3, ch3), S.enc3 = _block_fwd(m.enc3, p2, None, n, h3, w3, training, slots, att=m.att3)
    # bridge (dilated)
    (b, sa3), (S.br1, S.br2) = _pair_fwd(m.bridge[0], m.bridge[1], m.bridge[3], m.bridge[4], e3, None, n, h3, w3,
                                         training, 2, slots, gate=m.att3)
    # decoder with attention, virtual concat
    e3a, S.att3 = _att_fwd(m.att3, e3, b, n, hw3, early=ch3, sa=sa3)
    d3, S.dec3 = _block_fwd(m.dec3, b, e3a, n, h3, w3, training, slots)
    fuse_up = not training and not save   # inference: the decoder convs read up(d) without it being formed
    S.d3 = d3 if (training and _GATE_WGRAD_LOWRES) else None   # the gate's spatial weight gradient reads it
    # training: dec2.conv1 interpolates up(d3) itself as well (its forward stores the input split the weight
    # gradient reads, and the gate's weight gradient reads d3), so u3 is never formed (_TRAIN_UP3)
    u3, sa2 = _upsample_for_gate(d3, m.att2, n, h3, w3, h2, w2, m.dec2.conv1, e2.shape[1],
                                 fuse_up or (training and _TRAIN_UP3 and _GATE_WGRAD_LOWRES))
    e2a, S.att2 = _att_fwd(m.att2, e2, u3, n, hw2, early=ch2, sa=sa2)
    d2, S.dec2 = _block_fwd(m.dec2, u3, e2a, n, h2, w2, training, slots)
    S.d2 = d2 if (training and _GATE_WGRAD_LOWRES) else None
    u2, sa1 = _upsample_for_gate(d2, m.att1, n, h2, w2, h, w, m.dec1.conv1, e1.shape[1], fuse_up)
    e1a, S.att1 = _att_fwd(m.att1, e1, u2, n, hw1, early=ch1, sa=sa1)
    # multi-scale head + residual; dec1's output BN + ReLU is applied inside out_conv1's input
    # transform when out_conv1 keeps its input split (d1 itself is never written; _FUSE_D1 False: off)
    if _FUSE_D1 and _fuse_pair(m.out_conv1, training, w, 1):
        (d1, d1aff), S.dec1 = _block_fwd(m.dec1, u2, e1a, n, h, w, training, slots, activate=False)
    else:
        d1, S.dec1 = _block_fwd(m.dec1, u2, e1a, n, h, w, training, slots)
        d1aff = None
    # out_conv1 -> BN -> ReLU -> out_conv2 as a ConvBlock pair: out_bn1's BN + ReLU applied inside
    # out_conv2's input transform (train mode; out_conv2's dgrad and weight gradient run on h3 from
    # 32-channel-padded dy planes, so it keeps its input split)
    if _fuse_pair(m.out_conv2, training, w, 1):
        (o1, o1aff), S.out1 = _cbr_fwd(m.out_conv1, m.out_bn1, d1, None, n, h, w, training, 1, slots, in_affine=d1aff,
                                       activate=False)
        o2, S.out2 = _cbr_fwd(m.out_conv2, m.out_bn2, o1, None, n, h, w, training, 1, slots, in_affine=o1aff)
    else:
        o1, S.out1 = _cbr_fwd(m.out_conv1, m.out_bn1, d1, None, n, h, w, training, 1, slots, in_affine=d1aff)
        if (getattr(slots, "eval_epilogue", False) and _FUSE_HEAD and o1.shape[1] == 32
                and m.out_conv2.out_channels == 16 and H.h3_capable(32, 0, 16, w, 1)
                and H.query("srpde_conv_head_eval_supported", w)):
            # inference: out_conv2 -> out_bn2 -> ReLU -> final -> + residual in one pass (o2 never written)
            bn = m.out_bn2
            mean, invstd = _eval_stats(bn)
            wf = _fwd_weights(m.out_conv2, 32, 32, 0, w, 1)
            out = H.conv_head_eval(o1, wf, m.out_conv2.bias, mean, invstd, bn.weight, bn.bias, m.final.weight,
                                   m.final.bias, x, n, h, w)
            return out.view(n, 1, h, w), None
        o2, S.out2 = _cbr_fwd(m.out_conv2, m.out_bn2, o1, None, n, h, w, training, 1, slots)
    out = H.head_fwd(o2, m.final.weight, m.final.bias, x, n, hw1)
    if not save:
        return out.view(n, 1, h, w), None
    S.e1, S.e2, S.e3, S.b, S.u3, S.u2, S.o2 = e1, e2, e3, b, u3, u2, o2
    return out.view(n, 1, h, w), S


def unet_backward(m, S, dout, grads, grad_ready=None, wq=None, want_dx=False):
    """Reverse schedule.  ``grads``: param -> writable view (every one is fully written).
    ``want_dx``: also return the gradient w.r.t. the input x ([B, 3, H, W]; enc1.conv1's
    dgrad plus the residual's identity path into channel 0, models.py:74,101).
    ``grad_ready(group)`` is called as soon as a module group's gradients are queued (with
    ``wq``, a WgradStream, the weight gradients run on its side stream: a consumer waits for
    that stream too; the compute stream joins it before this returns)."""
    n, h, w = S.shape
    h2, w2, h3, w3 = h // 2, w // 2, h // 4, w // 4
    hw1, hw2, hw3 = h * w, h2 * w2, h3 * w3
    dev = dout.device
    P1, P2, P3 = n * hw1, n * hw2, n * hw3
    ready = grad_ready or (lambda g: None)
    slots = H.AmaxSlots(16, dev)   # max|dy| words of the 16 BN backward outputs
    dout = dout.contiguous().view(-1)
    # head
    do2 = H.empty(P1, 16, device=dev)
    H.head_bwd(dout, S.o2, m.final.weight, n, hw1, do2, grads[m.final.weight], grads[m.final.bias])
    _tap("o2", do2)
    ready("final")
    do1 = H.empty(P1, m.out_conv1.out_channels, device=dev)
    part = _cbr_bwd(m.out_conv2, m.out_bn2, S.out2, do2, n, h, w, 1, grads, slots, do1, below=(m.out_bn1, S.out1),
                    wq=wq)
    ready("out_bn2"); ready("out_conv2")
    _tap("o1", do1)
    dd1 = H.empty(P1, 64, device=dev)
    # out_conv1's dgrad writes dec1's output gradient: its epilogue also reduces dec1.bn2's backward
    part = _cbr_bwd(m.out_conv1, m.out_bn1, S.out1, do1, n, h, w, 1, grads, slots, dd1, part=part,
                    below=(m.dec1.bn2, S.dec1[1]), wq=wq)
    ready("out_bn1"); ready("out_conv1")
    _tap("d1", dd1)
    # dec1: grad of cat[u2 (128), e1a (64)]
    dcat1 = H.empty(P1, 192, device=dev)
    _block_bwd(m.dec1, S.dec1, dd1, n, h, w, grads, slots, dcat1, wq=wq, part=part)
    _tap("u2c", dcat1[:, :128])
    _tap("e1a", dcat1[:, 128:])
    ready("dec1")
    de1 = H.empty(P1, 64, device=dev)
    # the gating gradient (into dcat1[:, :128]) is folded into the upsample backward below; with the encoder-output
    # fusion the gate's input gradient is formed together with the max-pool backward into de1 (enc1's turn, below)
    fuse1 = _fuse_enc_out(S.enc1, 64, w)
    gate = _att_bwd(m.att1, S.att1, dcat1[:, 128:], S.e1, S.u2, n, hw1, grads, None if fuse1 else de1, False, None, True,
                    wq=wq, defer_dx=fuse1, g_lowres=(S.d2, h2, w2, h, w) if S.d2 is not None else None)
    if fuse1:
        gate, dm1 = gate
    ready("att1")
    dd2 = H.empty(P2, 128, device=dev)
    # dec2.bn2's backward reduction formed by the upsample backward that writes its output gradient
    part = H.upsample_bwd(dcat1[:, :128], dd2, n, h2, w2, h, w, False, gate=gate, bn=_up_bn(m.dec2, S.dec2))
    _tap("d2", dd2)
    # dec2: grad of cat[u3 (256), e2a (128)]
    dcat2 = H.empty(P2, 384, device=dev)
    _block_bwd(m.dec2, S.dec2, dd2, n, h2, w2, grads, slots, dcat2, wq=wq, part=part)
    _tap("u3c", dcat2[:, :256])
    _tap("e2a", dcat2[:, 256:])
    ready("dec2")
    de2 = H.empty(P2, 128, device=dev)
    # the gating gradient (into dcat2[:, :256]) is folded into the upsample backward below
    fuse2 = _fuse_enc_out(S.enc2, 128, w2)
    u3 = S.u3.x if isinstance(S.u3, H.UpsampledInput) else S.u3   # (the low-res rows: only g's width is read)
    gate = _att_bwd(m.att2, S.att2, dcat2[:, 256:], S.e2, u3, n, hw2, grads, None if fuse2 else de2, False, None,
                    True, wq=wq, defer_dx=fuse2, g_lowres=(S.d3, h3, w3, h2, w2) if S.d3 is not None else None)
    if fuse2:
        gate, dm2 = gate
    ready("att2")
    dd3 = H.empty(P3, 256, device=dev)
    part = H.upsample_bwd(dcat2[:, :256], dd3, n, h3, w3, h2, w2, False, gate=gate, bn=_up_bn(m.dec3, S.dec3))
    _tap("d3", dd3)
    # dec3: grad of cat[b (512), e3a (256)]
    dcat3 = H.empty(P3, 768, device=dev)
    _block_bwd(m.dec3, S.dec3, dd3, n, h3, w3, grads, slots, dcat3, wq=wq, part=part)
    _tap("e3a", dcat3[:, 512:])
    ready("dec3")
    de3 = H.empty(P3, 256, device=dev)
    bpart = None
    if _FUSE_GATING_BN:
        # the gating gradient into db = dcat3[:, :512] together with bridge[4]'s backward reduction
        gate = _att_bwd(m.att3, S.att3, dcat3[:, 512:], S.e3, S.b, n, hw3, grads, de3, False, None, True, wq=wq)
        _, _, yb, mb, ib, _, _ = S.br2
        bpart = H.gating_bn_reduce(gate[0], gate[1], dcat3[:, :512], yb, mb, ib, m.bridge[4].weight,
                                   m.bridge[4].bias)
    else:
        _att_bwd(m.att3, S.att3, dcat3[:, 512:], S.e3, S.b, n, hw3, grads, de3, False, dcat3[:, :512], True, wq=wq)
    _tap("b", dcat3[:, :512])
    ready("att3")
    # bridge: db = dcat3[:, :512]; its dgrad accumulates into de3
    dab1 = H.empty(P3, 512, device=dev)
    part = _cbr_bwd(m.bridge[3], m.bridge[4], S.br2, dcat3[:, :512], n, h3, w3, 2, grads, slots, dab1, part=bpart,
                    below=(m.bridge[1], S.br1), wq=wq)
    _tap("b1", dab1)
    _cbr_bwd(m.bridge[0], m.bridge[1], S.br1, dab1, n, h3, w3, 2, grads, slots, de3, True, part=part, wq=wq)
    _tap("e3", de3)
    ready("bridge")
    # encoder
    dp2 = H.empty(P3, 128, device=dev)
    _block_bwd(m.enc3, S.enc3, de3, n, h3, w3, grads, slots, dp2, wq=wq)
    ready("enc3")
    part = None
    if fuse2:
        part = _enc_out_bwd(m.enc2, S.enc2, S.att2, dcat2[:, 256:], dm2, S.e2, dp2, de2, n, h2, w2)
    else:
        H.maxpool_bwd(S.e2, dp2, de2, n, h2, w2, True)
    _tap("e2", de2)
    dp1 = H.empty(P2, 64, device=dev)
    _block_bwd(m.enc2, S.enc2, de2, n, h2, w2, grads, slots, dp1, wq=wq, part=part)
    ready("enc2")
    part = None
    if fuse1:
        part = _enc_out_bwd(m.enc1, S.enc1, S.att1, dcat1[:, 128:], dm1, S.e1, dp1, de1, n, h, w)
    else:
        H.maxpool_bwd(S.e1, dp1, de1, n, h, w, True)
    _tap("e1", de1)
    dx4 = H.empty(P1, S.x4.shape[1], device=dev) if want_dx else None
    _block_bwd(m.enc1, S.enc1, de1, n, h, w, grads, slots, dx4, wq=wq, part=part, last=True)
    ready("enc1")
    if wq is not None:
        wq.join()
    if dx4 is None:
        return None
    # NHWC [P, 4] -> NCHW [B, 3, H, W], and the residual x[:, 0:1] passes dout straight through
    dx = H.nhwc_to_nchw(dx4, n, 3, h, w)
    H.axpy_(dx, dout, channel=0, channels=3)
    return dx


class UNetFunction(torch.autograd.Function):
    """One autograd node for the whole network: forward/backward are the HIP schedules."""

    @staticmethod
    def forward(ctx, x, model, *params):
        out, saved = unet_forward(model, x, model.training, save=True)
        ctx.model = model
        ctx.saved = saved
        ctx.n_params = len(params)
        return out

    @staticmethod
    def backward(ctx, dout):
        model = ctx.model
        layout = model._flat_layout()
        total = layout[-1][2] + layout[-1][3]
        flat = torch.empty(total, dtype=torch.float32, device=dout.device)
        views = {p: flat[off:off + nn].view_as(p) for _, p, off, nn in layout}
        reducer = getattr(model, "_grad_reducer", None)
        ends = _group_end_offsets(layout)
        side = _WGRAD_STREAM and dout.is_cuda
        # with the weight gradients on a side stream, the dgrad chain may run on a high-priority
        # stream (_BWD_PRIORITY; on by default under data parallelism, see _BWD_PRIORITY)
        prio = _BWD_PRIORITY == "1" or (_BWD_PRIORITY == "auto" and reducer is not None)
        hi = _priority_stream(dout.device) if side and prio else None
        cur = torch.cuda.current_stream(dout.device) if dout.is_cuda else None
        if hi is not None:
            hi.wait_stream(cur)
        with torch.cuda.stream(hi) if hi is not None else contextlib.nullcontext():
            wq = WgradStream(dout.device) if side else None
            hook = None
            if reducer is not None:
                reducer.begin(flat, wait_streams=() if wq is None else (wq.side,))
                hook = lambda grp: reducer.ready(ends[grp])  # noqa: E731
            dx = unet_backward(model, ctx.saved, dout, views, hook, wq=wq, want_dx=ctx.needs_input_grad[0])
            if reducer is not None:
                reducer.finish()
        if hi is not None:
            cur.wait_stream(hi)
        ctx.saved = None
        grads = [views[p] for p in model._param_list()]
        return (dx, None, *grads)
