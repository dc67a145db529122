"""HIP MSE loss (reference ``nn.MSELoss()``, src/train_enhanced.py:70, :307).

``mse_loss`` keeps the loss scalar on the device (no host sync); its backward is the
HIP kernel dy = 2 (y - t) / numel * grad_out.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import hipops as H


class _MSEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y, t):
        y = y.contiguous()
        t = t.contiguous()
        ctx.save_for_backward(y, t)
        return H.mse_fwd(y, t)

    @staticmethod
    def backward(ctx, gout):
        y, t = ctx.saved_tensors
        dy = H.mse_bwd(y, t, gout.contiguous())
        return dy, None


def mse_loss(y: torch.Tensor, t: torch.Tensor) -> torch.Tensor:
    if y.shape != t.shape:
        raise ValueError(f"mse_loss: shape mismatch {tuple(y.shape)} vs {tuple(t.shape)}")
    if not y.is_cuda or y.dtype != torch.float32:
        raise RuntimeError("mse_loss: HIP path needs float32 ROCm tensors (no CPU fallback)")
    return _MSEFn.apply(y, t)


class MSELoss(nn.Module):
    """Drop-in for nn.MSELoss() with reduction='mean'."""

    def forward(self, input: torch.Tensor, target: torch.Tensor) -> torch.Tensor:  # noqa: A002
        return mse_loss(input, target)
