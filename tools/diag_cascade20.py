"""Bisect a change in the 20 -> 640 cascade's agreement with the reference fixture
(tests/test_gpu_cascade.py::test_cascade_20_to_640_matches_reference) over the executor switches."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)


def main():
    from state import fixture_state_torch
    from superresolution_for_pdes_amd import hipops as H, unet_exec as X
    from superresolution_for_pdes_amd.models import UNet
    from superresolution_for_pdes_amd.resolution_comparison import ml_multi_level_upscale, solve_multi_resolution
    z = np.load(os.path.join(ROOT, "tests", "golden", "cascade640_fixture.npz"))
    np.random.seed(0)
    data = solve_multi_resolution(20, [40, 80, 160, 320, 640])
    ref = z["ml640_from20"].astype(np.float64)
    base = {k: getattr(X, k) for k in ("_FUSE_ATT_APPLY", "_EVAL_EPI_F32", "_EVAL_STATS_CACHE", "_EVAL_EPI")}
    configs = [("default", {}, True, True), ("no att fusion", {"_FUSE_ATT_APPLY": False}, True, True),
               ("no f32 eval epilogue", {"_EVAL_EPI_F32": False}, True, True),
               ("no stats cache", {"_EVAL_STATS_CACHE": False}, True, True), ("h3 not h4", {}, False, True),
               ("no graphs", {}, True, False), ("no eval epilogues", {"_EVAL_EPI": False}, True, True),
               ("all off", {"_FUSE_ATT_APPLY": False, "_EVAL_EPI_F32": False, "_EVAL_STATS_CACHE": False}, False,
                False)]
    for name, sw, h4, graphs in configs:
        for k, v in base.items():
            setattr(X, k, sw.get(k, v))
        prev = H.set_h4(h4)
        m = UNet()
        m.load_state_dict(fixture_state_torch())
        m = m.cuda().eval()
        out = ml_multi_level_upscale(m, data, 640, "cuda", start_resolution=20, graphs=graphs)
        H.set_h4(prev)
        o80 = ml_multi_level_upscale(m, data, 40, "cuda", start_resolution=20, graphs=graphs)
        err = float(np.sqrt(np.mean((out[::3, ::5] - ref) ** 2)) / np.sqrt(np.mean(ref ** 2)))
        print(f"{name:22s} rel err {err:.3e}  level-1 out[0,:3] {np.array2string(o80[0, :3], precision=9)}",
              flush=True)


if __name__ == "__main__":
    main()
