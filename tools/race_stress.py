"""Determinism stress for single kernels under GPU sharing: every rank (process) repeats one op on
fixed inputs and compares each result with the first, bit for bit.  Run two or more processes on one
GPU (torch.distributed.run --nproc-per-node 2 tools/race_stress.py); no collectives are used."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from superresolution_for_pdes_amd import hipops as H  # noqa: E402

DEV = torch.device("cuda", 0)
rank = int(os.environ.get("RANK", "0"))
REPS = int(os.environ.get("STRESS_REPS", "40"))


def check(name, fn):
    ref = [t.clone() for t in fn()]
    bad = 0
    for _ in range(REPS):
        out = fn()
        if not all(torch.equal(a, b) for a, b in zip(ref, out)):
            bad += 1
    torch.cuda.synchronize()
    print(f"rank {rank} {name}: {bad}/{REPS} differ", flush=True)


def conv_case(n, c, cout, hw, dil, h3r):
    g = torch.Generator(device=DEV).manual_seed(c + cout)
    P = n * hw * hw
    x = torch.randn(P, c, device=DEV, generator=g).abs()
    x._srpde_amax = H.amax_of(x)
    w = torch.randn(cout, c, 3, 3, device=DEV, generator=g) * 0.05
    b = torch.randn(cout, device=DEV, generator=g)
    wf, _ = H.pack_conv_weights(w, c, True, False)
    H.set_h3r(h3r)

    def run():
        y = torch.empty(P, cout, device=DEV)
        st, _, _ = H.conv_stats_buffer(n, hw, hw, cout, DEV, c, 0, dil)
        xp = H.split_planes_buffer(P, c, DEV)
        H.conv_fwd(x, None, wf, b, y, n, hw, hw, cout, 3, dil, 1, False, st, xp)
        return y, st, xp
    check(f"conv c{c}->{cout} hw{hw} dil{dil} h3r={h3r}", run)


def main():
    torch.cuda.set_device(DEV)
    conv_case(64, 64, 64, 40, 1, True)
    conv_case(64, 64, 64, 40, 1, False)
    conv_case(64, 256, 512, 10, 2, False)
    conv_case(64, 128, 128, 20, 1, False)
    conv_case(64, 192, 64, 40, 1, True)


if __name__ == "__main__":
    main()
