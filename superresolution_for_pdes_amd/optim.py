"""Fused clip_grad_norm_ + AdamW on the HIP kernels (src/train_enhanced.py:74-75, :308).

``FusedAdamW`` is a ``torch.optim.Optimizer`` with AdamW's hyper-parameters and state
layout (``step`` / ``exp_avg`` / ``exp_avg_sq`` per parameter, so ``state_dict()`` has the
shape the reference checkpoints store at train_enhanced.py:120).  When the parameters
and their gradients are views of one flat buffer (``UNet.flatten_parameters_`` + the
executor's flat gradient), one norm reduction and one update launch cover all
7,834,588 parameters; the clip coefficient stays on the device.
"""
from __future__ import annotations

import torch

from . import hipops as H


def _flat_span(tensors):
    """If ``tensors`` tile one contiguous range of one storage in order, return a 1-D view of it."""
    if not tensors:
        return None
    t0 = tensors[0]
    if any(t is None for t in tensors):
        return None
    base = t0.data_ptr()
    off = 0
    for t in tensors:
        if not t.is_contiguous() or t.data_ptr() != base + 4 * off or t.untyped_storage().data_ptr() != \
                t0.untyped_storage().data_ptr():
            return None
        off += t.numel()
    start = (base - t0.untyped_storage().data_ptr()) // 4
    return torch.empty(0, dtype=t0.dtype, device=t0.device).set_(t0.untyped_storage(), start, (off,), (1,))


# bumped by every FusedAdamW.step: the update runs in a HIP kernel, which torch's tensor
# version counters do not see, so caches keyed on parameter values (unet_exec's eval-mode
# weight split) key on this as well
_STEPS = [0]


def step_count() -> int:
    return _STEPS[0]


class FusedAdamW(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, max_grad_norm=None):
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        self.max_grad_norm = max_grad_norm
        self.last_total_norm = None
        self._coef = None
        self._flat = {}

    def _group_buffers(self, gi, group):
        # memory order: the U-Net's flat buffer is laid out in backward-completion order
        params = sorted(group["params"], key=lambda t: t.data_ptr())
        key = gi
        fb = self._flat.get(key)
        fp = _flat_span(params)
        if fb is None or fb["fp"] is None or fp is None or fb["fp"].data_ptr() != fp.data_ptr() or \
                any(self.state[p].get("exp_avg") is None for p in params) or \
                _flat_span([self.state[p]["exp_avg"] for p in params]) is None:
            n = sum(p.numel() for p in params)
            m = torch.zeros(n, dtype=torch.float32, device=params[0].device)
            v = torch.zeros_like(m)
            off = 0
            step = None
            for p in params:
                st = self.state[p]
                if "exp_avg" in st:
                    m[off:off + p.numel()].copy_(st["exp_avg"].reshape(-1))
                    v[off:off + p.numel()].copy_(st["exp_avg_sq"].reshape(-1))
                if "step" in st and step is None:
                    step = st["step"]
                off += p.numel()
            step = torch.tensor(float(step) if step is not None else 0.0)
            off = 0
            for p in params:
                st = self.state[p]
                st["exp_avg"] = m[off:off + p.numel()].view_as(p)
                st["exp_avg_sq"] = v[off:off + p.numel()].view_as(p)
                st["step"] = step
                off += p.numel()
            fb = {"fp": fp, "m": m, "v": v, "step": step}
            self._flat[key] = fb
        return fb

    def state_dict(self):
        """torch.optim.AdamW's layout: every parameter's state holds its OWN ``step`` tensor (the
        fused path shares one counter internally; a shared tensor in a checkpoint would be
        incremented once per parameter by torch's AdamW after loading)."""
        sd = super().state_dict()
        sd["state"] = {k: {kk: (vv.clone() if kk == "step" and torch.is_tensor(vv) else vv) for kk, vv in v.items()}
                       for k, v in sd["state"].items()}
        return sd

    @torch.no_grad()
    def clip_grad_norm_(self, max_norm, grad_scale=1.0):
        """clip_grad_norm_(all params, max_norm) on device.  Like torch's, the NEXT step()
        uses the clipped gradients (the coefficient is applied inside the fused update
        instead of rewriting the gradients).  Returns the total-norm tensor (device), a fresh one per call
        as torch's is (a caller keeping a step's norm must not see the next step's)."""
        grads = [p.grad for g in self.param_groups for p in g["params"]]
        flat = _flat_span(sorted(grads, key=lambda t: t.data_ptr())) if all(g is not None for g in grads) else None
        if flat is None:
            flat = torch.cat([g.reshape(-1) for g in grads if g is not None])
        self._coef = torch.empty(2, dtype=torch.float32, device=flat.device)   # caching allocator: no launch
        H.clip_coef(flat, grad_scale, float(max_norm) if max_norm is not None else -1.0, self._coef)
        self._pending = True
        self.last_total_norm = self._coef[1]
        return self._coef[1]

    @torch.no_grad()
    def step(self, closure=None, grad_scale=1.0, max_grad_norm=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        mgn = max_grad_norm if max_grad_norm is not None else self.max_grad_norm
        if mgn is not None:
            self.clip_grad_norm_(mgn, grad_scale)
        coef = self._coef if getattr(self, "_pending", False) else None
        self._pending = False
        if coef is not None and coef.is_cuda:
            # the next clip_grad_norm_ replaces (frees) this buffer: if this step runs on another
            # stream than the one that allocated it, the caching allocator must not hand its memory
            # out again before this stream's update kernel has read it
            coef.record_stream(torch.cuda.current_stream(coef.device))
        _STEPS[0] += 1
        for gi, group in enumerate(self.param_groups):
            params = [p for p in group["params"] if p.grad is not None]
            if not params:
                continue
            b1, b2 = group["betas"]
            fb = self._group_buffers(gi, group)
            fb["step"] += 1
            step = int(fb["step"].item())
            gflat = _flat_span([p.grad for p in sorted(group["params"], key=lambda t: t.data_ptr())])
            if fb["fp"] is not None and gflat is not None:
                H.adamw_step(fb["fp"], gflat, fb["m"], fb["v"], group["lr"], b1, b2, group["eps"],
                             group["weight_decay"], step, coef, grad_scale)
            else:
                for p in params:
                    st = self.state[p]
                    H.adamw_step(p.data.view(-1), p.grad.contiguous().view(-1), st["exp_avg"].view(-1),
                                 st["exp_avg_sq"].view(-1), group["lr"], b1, b2, group["eps"],
                                 group["weight_decay"], step, coef, grad_scale)
        return loss
