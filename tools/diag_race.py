"""Locate a run-to-run difference in the train step's backward: the executor's debug taps (each
dgrad's dy split, dx, max|dx| slots and fused BN partials, in launch order) of R repeats of the same
step, compared with the first repeat.  Prints, per repeat, the first tap whose bits changed and how
many elements did.

    python tools/diag_race.py [R]
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests", "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)


def main():
    from branch import hip_step
    from state import fixture_state_torch
    from superresolution_for_pdes_amd import hipops as H, unet_exec as X
    from superresolution_for_pdes_amd.models import UNet
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    g = torch.Generator().manual_seed(4)
    x = torch.randn(16, 3, 40, 40, generator=g)
    x[:, 1] = 1.0
    t = torch.randn(16, 1, 40, 40, generator=g)
    for name, h4, stream in (("h4 + wgrad stream", True, True), ("h4 in line", True, False),
                             ("h3 + wgrad stream", False, True)):
        X._WGRAD_STREAM = stream
        prev = H.set_h4(h4)
        taps = []
        for _ in range(reps):
            m = UNet()
            m.load_state_dict(fixture_state_torch())
            m = m.cuda().train()
            m.flatten_parameters_()
            tp = {}
            hip_step(m, x.cuda(), t.cuda(), taps=tp)
            taps.append(tp)
        H.set_h4(prev)
        print(f"== {name}: {len(taps[0])} taps")
        for i, tp in enumerate(taps[1:], 1):
            first = None
            ndiff = 0
            for k, v in tp.items():
                r = taps[0][k]
                if not torch.equal(v.view(torch.uint8) if v.dtype != r.dtype else v, r):
                    ndiff += 1
                    if first is None:
                        d = (v.float() - r.float())
                        nz = int((d != 0).sum())
                        first = f"{k} shape {tuple(v.shape)} {nz} elems differ, max |d| {float(d.abs().max()):.3e}" \
                                f" (max |x| {float(r.float().abs().max()):.3e})"
                        if v.dim() >= 2 and nz:
                            idx = (d != 0).nonzero()[:4].tolist()
                            first += f" at {idx}"
            print(f"   repeat {i}: {ndiff} taps differ; first: {first}")
        sys.stdout.flush()


if __name__ == "__main__":
    main()
