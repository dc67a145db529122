"""Repeatability of the train step (forward + backward through the executor) on the GPU, per kernel
/ executor configuration: the same inputs and weights run R times must give the same bits.  Prints,
per configuration, the tensors whose bits changed between repeats and the branch-matched fp64
error of the first repeat's worst gradients (the bar of tests/test_gpu_unet.py's switch test).

    python tools/diag_determinism.py [R]          # DIAG_CONFIGS=default,... : a subset

Repeats after the first run with every torch.empty / empty_like result poisoned (NaN, then 1e30):
a kernel that reads memory it never wrote shows up as a tensor that changed under the poison.
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests", "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)


def main():
    from branch import hip_decisions, hip_step
    from oracle.unet_ref import clone_state, unet_forward as ref_fwd, trainable_names
    from state import fixture_state_torch
    from superresolution_for_pdes_amd import hipops as H, unet_exec as X
    from superresolution_for_pdes_amd.models import UNet
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    real_empty, real_empty_like = torch.empty, torch.empty_like
    poison = [None]

    def fill(t):
        if poison[0] is not None and t.is_cuda:
            if t.is_floating_point():
                t.fill_(poison[0] if t.dtype != torch.float16 or poison[0] != poison[0] else 6e4)
            elif t.dtype in (torch.int32, torch.int64):
                t.fill_(0x7f7f7f7f)
        return t

    torch.empty = lambda *a, **k: fill(real_empty(*a, **k))
    torch.empty_like = lambda *a, **k: fill(real_empty_like(*a, **k))
    g = torch.Generator().manual_seed(4)
    x = torch.randn(16, 3, 40, 40, generator=g)
    x[:, 1] = 1.0
    t = torch.randn(16, 1, 40, 40, generator=g)
    names = trainable_names()

    def oracle(dec, dtype):
        st = clone_state(fixture_state_torch(dtype))
        for n_ in names:
            st[n_].requires_grad_(True)
        out = ref_fwd(st, x.to(dtype), True, decisions=dec)
        torch.nn.functional.mse_loss(out, t.to(dtype)).backward()
        return {n_: st[n_].grad.double() for n_ in names}

    base = {k: getattr(X, k) for k in ("_FUSE_ATT_APPLY", "_WGRAD_STREAM", "_PRESPLIT_BWD")}
    configs = [("default", {}, True), ("h3 not h4", {}, False), ("no att fusion", {"_FUSE_ATT_APPLY": False}, True),
               ("no wgrad stream", {"_WGRAD_STREAM": False}, True),
               ("h3, no att fusion, no stream", {"_FUSE_ATT_APPLY": False, "_WGRAD_STREAM": False}, False)]
    if os.environ.get("DIAG_CONFIGS"):
        keep = os.environ["DIAG_CONFIGS"].split(",")
        configs = [c for c in configs if c[0] in keep]
    for name, sw, h4 in configs:
        for k, v in base.items():
            setattr(X, k, sw.get(k, v))
        prev = H.set_h4(h4)
        runs = []
        for r_ in range(reps):
            poison[0] = (None, float("nan"), 1e30)[r_ % 3]
            m = UNet()
            m.load_state_dict(fixture_state_torch())
            m = m.cuda().train()
            m.flatten_parameters_()
            out, grads, dx, S = hip_step(m, x.cuda(), t.cuda())
            poison[0] = None
            runs.append((out.clone(), {k: v.clone() for k, v in grads.items()}, dx.clone(), hip_decisions(m, S)))
        H.set_h4(prev)
        changed = []
        for i, r in enumerate(runs[1:], 1):
            if not torch.equal(r[0], runs[0][0]):
                changed.append((f"[{i}] out", float((r[0] - runs[0][0]).abs().max())))
            if not torch.equal(r[2], runs[0][2]):
                changed.append((f"[{i}] dx", float((r[2] - runs[0][2]).abs().max())))
            for n_ in names:
                if not torch.equal(r[1][n_], runs[0][1][n_]):
                    changed.append((f"[{i}] {n_}",
                                    float((r[1][n_] - runs[0][1][n_]).norm() / runs[0][1][n_].norm())))
        g64, g32 = oracle(runs[0][3], torch.float64), oracle(runs[0][3], torch.float32)
        errs = []
        for n_ in names:
            e = float((runs[0][1][n_].double().cpu() - g64[n_]).norm() / g64[n_].norm())
            e32 = float((g32[n_] - g64[n_]).norm() / g64[n_].norm())
            errs.append((e / max(1e-4, 3 * e32), n_, e, e32))
        errs.sort(reverse=True)
        print(f"== {name}: {len(changed)} changed tensors over {reps} repeats {sorted(set(c[0] for c in changed))[:8]}")
        for c in changed[:12]:
            print(f"   changed {c[0]} {c[1]:.3e}")
        for r, n_, e, e32 in errs[:4]:
            print(f"   err/bar {r:.2f} {n_} {e:.3e} (ref fp32 {e32:.3e})")
        sys.stdout.flush()
    for k, v in base.items():
        setattr(X, k, v)


if __name__ == "__main__":
    main()
