"""Functional torch-CPU restatement of the reference attention U-Net.

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``): the checker for the HIP path
and the timed ``cpu_baseline`` in ``bench.py``.  It never runs inside the product.

Restates, op for op, reference ``src/models.py``:

* ``ConvBlock.forward``       models.py:21-24   conv3x3 p1 -> BN -> ReLU, twice
* ``UNet.__init__/forward``   models.py:27-101  encoder / dilated bridge / attention
                                                 decoder / head / residual
* ``AttentionGate.forward``   models.py:119-130 channel gate x spatial gate
* ``init_weights``            models.py:209-222 (``kaiming_init_state``)

and the inner training step of ``src/train_enhanced.py:68-75`` (MSE, backward,
clip_grad_norm_, AdamW) in ``train_step``.

Parameters live in a plain ``dict[name -> Tensor]`` keyed by the reference's
state-dict names (``param_specs``), so the same dict can be loaded into either the
reference module or the HIP module.  Works in float32 or float64 (pass tensors of
the wanted dtype).
"""
from __future__ import annotations

import math
from collections import OrderedDict

import torch
import torch.nn.functional as F

BN_EPS = 1e-5        # nn.BatchNorm2d default (models.py:17,19,44,47,58,60)
BN_MOMENTUM = 0.1    # nn.BatchNorm2d default


# ----------------------------------------------------------------------------------
# Architecture table (reference models.py:36-70).  Order == reference state_dict order.
# ----------------------------------------------------------------------------------
def _conv(name, cin, cout, k):
    return [(f"{name}.weight", (cout, cin, k, k), "conv_w"), (f"{name}.bias", (cout,), "conv_b")]


def _bn(name, c):
    return [(f"{name}.weight", (c,), "bn_w"), (f"{name}.bias", (c,), "bn_b"),
            (f"{name}.running_mean", (c,), "bn_rm"), (f"{name}.running_var", (c,), "bn_rv"),
            (f"{name}.num_batches_tracked", (), "bn_nbt")]


def _block(name, cin, cout):
    return (_conv(f"{name}.conv1", cin, cout, 3) + _bn(f"{name}.bn1", cout)
            + _conv(f"{name}.conv2", cout, cout, 3) + _bn(f"{name}.bn2", cout))


def _att(name, c, g, reduction=8):
    return (_conv(f"{name}.channel_attention.1", c, c // reduction, 1)
            + _conv(f"{name}.channel_attention.3", c // reduction, c, 1)
            + _conv(f"{name}.spatial_attention.0", g, 1, 1))


def param_specs(in_channels: int = 3):
    """[(state_dict_name, shape, kind)] in reference ``UNet().state_dict()`` order."""
    s = []
    s += _block("enc1", in_channels, 64) + _block("enc2", 64, 128) + _block("enc3", 128, 256)
    s += _conv("bridge.0", 256, 512, 3) + _bn("bridge.1", 512)
    s += _conv("bridge.3", 512, 512, 3) + _bn("bridge.4", 512)
    s += _block("dec3", 512 + 256, 256) + _block("dec2", 256 + 128, 128) + _block("dec1", 128 + 64, 64)
    s += _conv("out_conv1", 64, 32, 3) + _bn("out_bn1", 32)
    s += _conv("out_conv2", 32, 16, 3) + _bn("out_bn2", 16)
    s += _conv("final", 16, 1, 1)
    s += _att("att3", 256, 512) + _att("att2", 128, 256) + _att("att1", 64, 128)
    return s


def trainable_names(in_channels: int = 3):
    return [n for n, _, k in param_specs(in_channels) if k in ("conv_w", "conv_b", "bn_w", "bn_b")]


def kaiming_init_state(seed: int = 0, in_channels: int = 3, dtype=torch.float32):
    """Restates ``init_weights`` (models.py:209-222): conv kaiming_normal_(fan_out, relu),
    conv bias 0, BN gamma 1 / beta 0; fresh BN buffers."""
    g = torch.Generator().manual_seed(seed)
    st = OrderedDict()
    for name, shape, kind in param_specs(in_channels):
        if kind == "conv_w":
            fan_out = shape[0] * shape[2] * shape[3]
            st[name] = torch.randn(shape, generator=g, dtype=torch.float64).mul_(math.sqrt(2.0 / fan_out)).to(dtype)
        elif kind in ("conv_b", "bn_b", "bn_rm"):
            st[name] = torch.zeros(shape, dtype=dtype)
        elif kind in ("bn_w", "bn_rv"):
            st[name] = torch.ones(shape, dtype=dtype)
        else:
            st[name] = torch.zeros((), dtype=torch.int64)
    return st


# ----------------------------------------------------------------------------------
# Forward
# ----------------------------------------------------------------------------------
def _bn_apply(st, name, x, training):
    """nn.BatchNorm2d.forward (train: batch stats + running update; eval: running stats)."""
    if training:
        st[f"{name}.num_batches_tracked"] = st[f"{name}.num_batches_tracked"] + 1
    return F.batch_norm(x, st[f"{name}.running_mean"], st[f"{name}.running_var"],
                        st[f"{name}.weight"], st[f"{name}.bias"], training, BN_MOMENTUM, BN_EPS)


def _conv_apply(st, name, x, padding=0, dilation=1):
    return F.conv2d(x, st[f"{name}.weight"], st[f"{name}.bias"], padding=padding, dilation=dilation)


def _relu(z, decisions, key):
    """F.relu / nn.ReLU; with ``decisions`` (see unet_forward) the ReLU takes the given branch
    mask instead of deciding from its own (fp64) input: relu(z) := z * mask."""
    if decisions is None:
        return F.relu(z)
    return z * decisions[key].to(device=z.device, dtype=z.dtype)


def _maxpool(x, decisions, key):
    """F.max_pool2d(x, 2); with ``decisions`` the window maxima are taken at the given argmax
    indices (max_pool2d_with_indices layout: flat h*W+w per channel plane)."""
    if decisions is None:
        return F.max_pool2d(x, 2)
    idx = decisions[key].to(x.device)
    n, c, h2, w2 = idx.shape
    return x.flatten(2).gather(2, idx.flatten(2)).view(n, c, h2, w2)


def conv_block(st, name, x, training, decisions=None):
    """ConvBlock.forward, models.py:21-24."""
    x = _relu(_bn_apply(st, f"{name}.bn1", _conv_apply(st, f"{name}.conv1", x, 1), training), decisions,
              f"{name}.bn1")
    x = _relu(_bn_apply(st, f"{name}.bn2", _conv_apply(st, f"{name}.conv2", x, 1), training), decisions,
              f"{name}.bn2")
    return x


def attention_gate(st, name, x, gating, decisions=None, tap=None):
    """AttentionGate.forward, models.py:119-130.  ``tap``: receives the spatial pre-activation
    (``<name>.sa_pre``), whose gradient summed over the pixels is the spatial bias gradient."""
    m = x.mean(dim=(2, 3), keepdim=True)                                  # AdaptiveAvgPool2d(1)
    h = _relu(_conv_apply(st, f"{name}.channel_attention.1", m), decisions, f"{name}.channel_attention.2")
    ca = torch.sigmoid(_conv_apply(st, f"{name}.channel_attention.3", h))
    x = x * ca
    if gating.shape[-2:] != x.shape[-2:]:                                  # models.py:125-126
        gating = F.interpolate(gating, size=x.shape[-2:], mode="bilinear", align_corners=True)
    pre = _conv_apply(st, f"{name}.spatial_attention.0", gating)
    if tap is not None:
        tap(f"{name}.sa_pre", pre)
    sa = torch.sigmoid(pre)
    return x * sa


def up2(x):
    """nn.Upsample(scale_factor=2, mode='bilinear', align_corners=True), models.py:70."""
    return F.interpolate(x, scale_factor=2, mode="bilinear", align_corners=True)


def unet_forward(st, x, training: bool, taps=None, decisions=None):
    """UNet.forward, models.py:72-101.  ``st`` running stats are updated in place
    (functionally: the dict entries are replaced) when ``training``.  ``taps`` (a dict, for
    diagnostics): receives the named intermediates with ``retain_grad()`` so their gradients
    can be compared stage by stage (tools/diag_stages.py).

    ``decisions`` (optional): the discrete choices of another implementation's forward -- the
    ReLU masks after every BatchNorm (key: the BN's name) and in the channel attention (key
    ``att*.channel_attention.2``), and the max-pool argmax indices (``pool1``, ``pool2``).  The
    oracle then evaluates the SAME branch of the piecewise-smooth network in its own precision:
    an fp32 implementation and fp64 disagree on a ReLU whose input is within rounding of 0,
    and a single such flip moves an activation gradient by ~1/sqrt(numel) in relative L2 (it
    is what limits the reference's own fp32-vs-fp64 agreement); on a shared branch the
    remaining difference is arithmetic error only."""
    def tap(name, t):
        if taps is not None and t.requires_grad:
            t.retain_grad()
            taps[name] = t
        return t
    coarse = x[:, 0:1]
    D = decisions
    e1 = tap("e1", conv_block(st, "enc1", x, training, D))
    e2 = tap("e2", conv_block(st, "enc2", _maxpool(e1, D, "pool1"), training, D))
    e3 = tap("e3", conv_block(st, "enc3", _maxpool(e2, D, "pool2"), training, D))
    b = tap("b1", _relu(_bn_apply(st, "bridge.1", _conv_apply(st, "bridge.0", e3, 2, 2), training), D, "bridge.1"))
    b = tap("b", _relu(_bn_apply(st, "bridge.4", _conv_apply(st, "bridge.3", b, 2, 2), training), D, "bridge.4"))
    e3a = tap("e3a", attention_gate(st, "att3", e3, b, D, tap))
    d3 = tap("d3", conv_block(st, "dec3", torch.cat([b, e3a], 1), training, D))
    e2a = tap("e2a", attention_gate(st, "att2", e2, tap("u3g", up2(d3)), D, tap))
    d2 = tap("d2", conv_block(st, "dec2", torch.cat([tap("u3c", up2(d3)), e2a], 1), training, D))
    e1a = tap("e1a", attention_gate(st, "att1", e1, tap("u2g", up2(d2)), D, tap))
    d1 = tap("d1", conv_block(st, "dec1", torch.cat([tap("u2c", up2(d2)), e1a], 1), training, D))
    y = tap("o1", _relu(_bn_apply(st, "out_bn1", _conv_apply(st, "out_conv1", d1, 1), training), D, "out_bn1"))
    y = tap("o2", _relu(_bn_apply(st, "out_bn2", _conv_apply(st, "out_conv2", y, 1), training), D, "out_bn2"))
    y = _conv_apply(st, "final", y)
    return y + coarse


def clone_state(st, dtype=None):
    out = OrderedDict()
    for k, v in st.items():
        v = v.detach().clone()
        if dtype is not None and v.is_floating_point():
            v = v.to(dtype)
        out[k] = v
    return out


def forward_with_grads(st, x, target, training=True, decisions=None):
    """One MSE forward/backward (train_enhanced.py:69-72).  Returns (out, loss, grads, st')."""
    st = clone_state(st)
    names = [n for n in trainable_names() if n in st]
    for n in names:
        st[n].requires_grad_(True)
    out = unet_forward(st, x, training, decisions=decisions)
    loss = F.mse_loss(out, target)                           # nn.MSELoss(), train_enhanced.py:307
    grads = torch.autograd.grad(loss, [st[n] for n in names])
    return out.detach(), loss.detach(), OrderedDict(zip(names, [g.detach() for g in grads])), st


def train_step(st, x, target, lr=2e-4, weight_decay=1e-4, grad_clip=1.0, opt_state=None, step=1):
    """train_enhanced.py:68-75: zero_grad, forward, MSE, backward, clip_grad_norm_(1.0),
    AdamW(lr=2e-4, wd=1e-4) step.  Returns (loss, new_state, grads, opt_state)."""
    out, loss, grads, st = forward_with_grads(st, x, target, True)
    names = list(grads.keys())
    params = [st[n].detach().clone() for n in names]
    gl = [grads[n].clone() for n in names]
    total = torch.norm(torch.stack([torch.norm(g, 2.0) for g in gl]), 2.0)  # clip_grad_norm_
    coef = torch.clamp(grad_clip / (total + 1e-6), max=1.0)
    gl = [g * coef for g in gl]
    if opt_state is None:
        opt_state = {n: (torch.zeros_like(p), torch.zeros_like(p)) for n, p in zip(names, params)}
    b1, b2, eps = 0.9, 0.999, 1e-8
    new = OrderedDict(st)
    for n, p, g in zip(names, params, gl):
        m, v = opt_state[n]
        p = p * (1 - lr * weight_decay)                                   # decoupled weight decay
        m = m * b1 + g * (1 - b1)
        v = v * b2 + g * g * (1 - b2)
        bc1 = 1 - b1 ** step
        bc2 = 1 - b2 ** step
        denom = (v.sqrt() / math.sqrt(bc2)) + eps
        p = p - (lr / bc1) * m / denom
        opt_state[n] = (m, v)
        new[n] = p
    for k in new:
        new[k] = new[k].detach()
    return loss, new, grads, opt_state, total
