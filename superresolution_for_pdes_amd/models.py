"""Drop-in for reference ``src/models.py`` on MI355X.

Same classes, constructor signatures and state-dict keys as the reference
(``ConvBlock`` models.py:6-24, ``UNet`` :26-101, ``AttentionGate`` :103-130,
``PDEDataset`` :132-207, ``init_weights`` :209-222).  Parameters stay owned by
``nn.Conv2d`` / ``nn.BatchNorm2d`` children (so ``torch.load(...)['model_state_dict']``
from reference checkpoints round-trips: 132 keys), but every composite ``forward`` --
``UNet``, ``ConvBlock``, ``AttentionGate`` -- and its backward run as hand-written HIP
kernels from ``libsrpde_hip.so``; the leaf Conv2d/BatchNorm2d modules are parameter
containers and are never called on the hot path.  There is no CPU fallback: on a host
without a ROCm device these forwards raise.
"""
from __future__ import annotations

from typing import Tuple

import torch
import torch.nn as nn

from . import hipops as H
from . import unet_exec as X


# ------------------------------ NCHW <-> [P, C] views --------------------------------
def _rows_view(x):
    """[N,C,H,W] tensor whose memory is NHWC with a uniform pixel stride -> [P, C] view, else None."""
    n, c, h, w = x.shape
    if c % 4 or x.dtype != torch.float32 or not x.is_cuda:
        return None
    sn, sc, sh, sw = x.stride()
    if sc != 1 or sw % 4 or sh != w * sw or sn != h * sh or (x.data_ptr() % 16):
        return None
    return x.as_strided((n * h * w, c), (sw, 1))


def _to_rows(x):
    """Model-boundary staging: NCHW / channels-last input -> NHWC [P, Cpad] (Cpad = ceil4(C))."""
    if not x.is_cuda or x.dtype != torch.float32:
        raise RuntimeError("HIP path needs a float32 tensor on a ROCm device (no CPU fallback)")
    r = _rows_view(x)
    if r is not None:
        return r
    c = x.shape[1]
    return H.nchw_to_nhwc(x.contiguous(), (c + 3) // 4 * 4)


def _from_rows(r, n, c, h, w):
    """[P, >=C] rows -> logical [N, C, H, W] (channels-last strides, no copy)."""
    return r[:, :c].as_strided((n, c, h, w), (h * w * r.stride(0), 1, w * r.stride(0), r.stride(0)))


class ConvBlock(nn.Module):
    def __init__(self, in_channels: int, out_channels: int):
        """Double conv3x3(p=1) -> BatchNorm2d -> ReLU (reference models.py:6-24)."""
        super().__init__()
        self.conv1 = nn.Conv2d(in_channels, out_channels, kernel_size=3, padding=1)
        self.bn1 = nn.BatchNorm2d(out_channels)
        self.conv2 = nn.Conv2d(out_channels, out_channels, kernel_size=3, padding=1)
        self.bn2 = nn.BatchNorm2d(out_channels)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        params = [self.conv1.weight, self.conv1.bias, self.bn1.weight, self.bn1.bias,
                  self.conv2.weight, self.conv2.bias, self.bn2.weight, self.bn2.bias]
        if torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in params)):
            return _ConvBlockFn.apply(x, self, *params)
        n, _, h, w = x.shape
        a, _ = X._block_fwd(self, _to_rows(x), None, n, h, w, self.training, H.AmaxSlots(2, x.device))
        return _from_rows(a, n, self.conv2.out_channels, h, w)


class _ConvBlockFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, blk, *params):
        n, c, h, w = x.shape
        xr = _to_rows(x)
        a, saved = X._block_fwd(blk, xr, None, n, h, w, blk.training, H.AmaxSlots(2, x.device))
        ctx.blk, ctx.saved, ctx.shape, ctx.cin, ctx.cpad = blk, saved, (n, h, w), c, xr.shape[1]
        return _from_rows(a, n, blk.conv2.out_channels, h, w)

    @staticmethod
    def backward(ctx, dout):
        blk = ctx.blk
        n, h, w = ctx.shape
        # eval mode is handled inside (the BN backward drops its batch-statistic terms)
        da = _to_rows(dout)
        params = [blk.conv1.weight, blk.conv1.bias, blk.bn1.weight, blk.bn1.bias,
                  blk.conv2.weight, blk.conv2.bias, blk.bn2.weight, blk.bn2.bias]
        grads = {p: torch.empty_like(p) for p in params}
        dx = H.empty(n * h * w, ctx.cpad, device=dout.device) if ctx.needs_input_grad[0] else None
        X._block_bwd(blk, ctx.saved, da, n, h, w, grads, H.AmaxSlots(2, dout.device), dx)
        gx = _from_rows(dx, n, ctx.cin, h, w) if dx is not None else None
        return (gx, None, *[grads[p] for p in params])


class UNet(nn.Module):
    def __init__(self, in_channels: int = 3):
        """Attention U-Net for 20->40 PDE super-resolution (reference models.py:26-70)."""
        super().__init__()
        if in_channels != 3:
            raise ValueError("the reference forward splits channel 0 as the coarse solution; in_channels=3")
        self.enc1 = ConvBlock(in_channels, 64)
        self.enc2 = ConvBlock(64, 128)
        self.enc3 = ConvBlock(128, 256)
        self.bridge = nn.Sequential(
            nn.Conv2d(256, 512, kernel_size=3, padding=2, dilation=2),
            nn.BatchNorm2d(512),
            nn.ReLU(),
            nn.Conv2d(512, 512, kernel_size=3, padding=2, dilation=2),
            nn.BatchNorm2d(512),
            nn.ReLU(),
        )
        self.dec3 = ConvBlock(512 + 256, 256)
        self.dec2 = ConvBlock(256 + 128, 128)
        self.dec1 = ConvBlock(128 + 64, 64)
        self.out_conv1 = nn.Conv2d(64, 32, kernel_size=3, padding=1)
        self.out_bn1 = nn.BatchNorm2d(32)
        self.out_conv2 = nn.Conv2d(32, 16, kernel_size=3, padding=1)
        self.out_bn2 = nn.BatchNorm2d(16)
        self.final = nn.Conv2d(16, 1, kernel_size=1)
        self.att3 = AttentionGate(256, 512)
        self.att2 = AttentionGate(128, 256)
        self.att1 = AttentionGate(64, 128)
        self.pool = nn.MaxPool2d(2)
        self.up = nn.Upsample(scale_factor=2, mode="bilinear", align_corners=True)
        self._layout_cache = None
        self._flat_params = None
        self._grad_reducer = None
        for name, mod in self.named_modules():
            object.__setattr__(mod, "_srpde_name", name)

    # -- flat parameter storage (one contiguous buffer in backward-completion order) --
    def _flat_layout(self):
        if self._layout_cache is None:
            self._layout_cache = X.flat_layout(self)
        return self._layout_cache

    def _param_list(self):
        return [p for _, p in self.named_parameters()]

    def flatten_parameters_(self):
        """Re-home every parameter as a view of one flat device buffer (no-op if already)."""
        layout = self._flat_layout()
        total = layout[-1][2] + layout[-1][3]
        fp = self._flat_params
        dev = layout[0][1].device
        ok = (fp is not None and fp.device == dev and
              all(p.data_ptr() == fp.data_ptr() + 4 * off for _, p, off, _ in layout))
        if ok:
            return fp
        fp = torch.empty(total, dtype=torch.float32, device=dev)
        with torch.no_grad():
            for _, p, off, n in layout:
                fp[off:off + n].copy_(p.detach().reshape(-1))
                p.data = fp[off:off + n].view_as(p)
        self._flat_params = fp
        return fp

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        """UNet.forward (reference models.py:72-101) on the HIP schedule of unet_exec."""
        if x.is_cuda:
            self.flatten_parameters_()
        params = self._param_list()
        if torch.is_grad_enabled() and any(p.requires_grad for p in params):
            return X.UNetFunction.apply(x, self, *params)
        return X.unet_forward(self, x, self.training)[0]


class AttentionGate(nn.Module):
    def __init__(self, in_channels: int, gating_channels: int, reduction: int = 8):
        """Channel x spatial attention gate (reference models.py:103-130)."""
        super().__init__()
        if reduction != 8:
            raise ValueError("HIP attention kernels implement reduction=8 (the reference value)")
        self.channel_attention = nn.Sequential(
            nn.AdaptiveAvgPool2d(1),
            nn.Conv2d(in_channels, in_channels // reduction, 1),
            nn.ReLU(inplace=True),
            nn.Conv2d(in_channels // reduction, in_channels, 1),
            nn.Sigmoid(),
        )
        self.spatial_attention = nn.Sequential(
            nn.Conv2d(gating_channels, 1, kernel_size=1),
            nn.Sigmoid(),
        )

    def forward(self, x: torch.Tensor, gating: torch.Tensor) -> torch.Tensor:
        params = list(self.parameters())
        if torch.is_grad_enabled() and (x.requires_grad or gating.requires_grad or
                                        any(p.requires_grad for p in params)):
            return _AttentionFn.apply(x, gating, self, *params)
        out, _ = _att_forward(self, x, gating)
        return out


def _att_forward(att, x, gating):
    n, c, h, w = x.shape
    xr = _to_rows(x)
    gr = _to_rows(gating)
    gh, gw = gating.shape[-2:]
    resized = (gh, gw) != (h, w)
    if resized:  # models.py:125-126
        gr = H.upsample_fwd(gr, n, gh, gw, h, w)
    out, saved = X._att_fwd(att, xr, gr, n, h * w)
    return _from_rows(out, n, c, h, w), (xr, gr, saved, resized, (gh, gw), gating.shape[1])


class _AttentionFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gating, att, *params):
        out, st = _att_forward(att, x, gating)
        ctx.att, ctx.st, ctx.shape = att, st, tuple(x.shape)
        return out

    @staticmethod
    def backward(ctx, dout):
        att = ctx.att
        xr, gr, saved, resized, (gh, gw), gc = ctx.st
        n, c, h, w = ctx.shape
        params = list(att.parameters())
        grads = {p: torch.empty_like(p) for p in params}
        dx = H.empty(n * h * w, xr.shape[1], device=dout.device)
        dg = H.empty(n * h * w, gr.shape[1], device=dout.device)
        X._att_bwd(att, saved, _to_rows(dout), xr, gr, n, h * w, grads, dx, False, dg, False)
        if resized:
            dg0 = H.empty(n * gh * gw, gr.shape[1], device=dout.device)
            H.upsample_bwd(dg, dg0, n, gh, gw, h, w, False)
            dg, hh, ww = dg0, gh, gw
        else:
            hh, ww = h, w
        return (_from_rows(dx, n, c, h, w), _from_rows(dg, n, gc, hh, ww), None, *[grads[p] for p in params])


class PDEDataset(torch.utils.data.Dataset):
    def __init__(self, data_dict: dict, device: str = "cuda"):
        """Normalised (coarse-upsampled, theta, f) -> u_fine pairs (reference models.py:132-203).

        Statistics follow the reference exactly: fp32 mean / unbiased std over the whole
        split, theta passed through when std < 1e-6, coarse normalised with the FINE
        statistics, then bilinear (align_corners=True) to the fine grid -- normalisation,
        resize and channel stack run as one HIP pass (srpde_pde_dataset_assemble).  Tensors
        live on ``device``; batches are gathered by index on the device (``batch(idx)``), no
        DataLoader workers needed.
        """
        self.device = device
        if not str(device).startswith("cuda"):
            raise RuntimeError("PDEDataset keeps its tensors on a ROCm device (the HIP path has no CPU fallback)")
        f32 = lambda a: torch.as_tensor(a).to(device=device, dtype=torch.float32)  # noqa: E731
        self.u_coarse = f32(data_dict["u_coarse"])
        self.u_fine = f32(data_dict["u_fine"])
        self.f_fine = f32(data_dict["f_fine"])
        self.theta_fine = f32(data_dict["theta_fine"])
        self.has_subdomain_flag = "is_subdomain" in data_dict
        if self.has_subdomain_flag:
            self.is_subdomain = torch.as_tensor(data_dict["is_subdomain"]).bool().to(device)
        self.u_mean = self.u_fine.mean()
        self.u_std = self.u_fine.std()
        self.f_mean = self.f_fine.mean()
        self.f_std = self.f_fine.std()
        self.theta_is_constant = bool(self.theta_fine.std() < 1e-6)
        if self.theta_is_constant:
            self.theta_mean, self.theta_std = 0, 1
            print("Detected constant theta field, skipping normalization")
        else:
            self.theta_mean = self.theta_fine.mean()
            self.theta_std = self.theta_fine.std()
        # normalisation, the coarse field's resize to the fine grid and the channel stack in one
        # HIP pass (srpde_pde_dataset_assemble); model-ready inputs [N, 3, nf, nf], targets [N, 1, nf, nf]
        one, zero = torch.ones((), device=device), torch.zeros((), device=device)
        tm = zero if self.theta_is_constant else self.theta_mean
        ts = one if self.theta_is_constant else self.theta_std
        stats = torch.stack([self.u_mean, self.u_std, self.f_mean, self.f_std, tm, ts]).float().contiguous()
        self.inputs, self.targets = H.pde_dataset_assemble(self.u_coarse.contiguous(), self.u_fine.contiguous(),
                                                           self.theta_fine.contiguous(), self.f_fine.contiguous(),
                                                           stats, self.theta_is_constant)

    # the reference's intermediate fields (models.py:170-187), as views of the assembled tensors
    @property
    def u_fine_norm(self):
        return self.targets[:, 0]

    @property
    def u_coarse_norm(self):
        return (self.u_coarse - self.u_mean) / self.u_std

    @property
    def f_fine_norm(self):
        return self.inputs[:, 2]

    @property
    def theta_fine_norm(self):
        return self.inputs[:, 1]

    @property
    def u_coarse_upsampled(self):
        return self.inputs[:, 0:1]

    def __len__(self) -> int:
        return len(self.u_fine)

    def __getitem__(self, idx: int) -> Tuple[torch.Tensor, torch.Tensor]:
        return self.inputs[idx], self.targets[idx]

    def batch(self, idx):
        return self.inputs.index_select(0, idx), self.targets.index_select(0, idx)

    def denormalize(self, x: torch.Tensor) -> torch.Tensor:
        return x * self.u_std + self.u_mean


def upsample_bilinear(x, ho, wo):
    """F.interpolate(x, (ho, wo), mode='bilinear', align_corners=True) on the HIP kernel.

    x: [N, 1, h, w] CUDA fp32 -> [N, 1, ho, wo].  With one channel NCHW == NHWC, so the
    field is handed to the kernel as-is (scalar-channel variant)."""
    n, c, h, w = x.shape
    if c != 1:
        raise ValueError("upsample_bilinear: single-channel fields only")
    xr = x.contiguous().view(n * h * w, 1)
    out = H.upsample_fwd(xr, n, h, w, ho, wo)
    return out.view(n, 1, ho, wo)


def init_weights(m: nn.Module):
    """Kaiming-normal(fan_out, relu) conv weights, zero biases, BN gamma=1 / beta=0
    (reference models.py:209-222)."""
    if isinstance(m, nn.Conv2d):
        nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
        if m.bias is not None:
            nn.init.constant_(m.bias, 0)
    elif isinstance(m, nn.BatchNorm2d):
        nn.init.constant_(m.weight, 1)
        nn.init.constant_(m.bias, 0)
