"""Cross-check of a TRAINED model's cascade against the REAL reference (build container only).

tools/e2e_accuracy.py --save DIR (on the GPU box) trains with the reference config on
device-generated data and saves the best weights plus its HIP cascade outputs for test field
seed 0 (solve_multi_resolution(40, [80..640]) after np.random.seed(0)).  This script loads those
weights into the reference's own UNet (src/models.py) and runs the reference's
solve_multi_resolution + ml_multi_level_upscale (src/resolution_comparison.py:13-229) on CPU
fp32, then compares the physical fields: the north-star bar is RMSE <= 1e-5.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/crosscheck_trained_cascade.py DIR OUT.json
"""
import json
import os
import sys
import types

import numpy as np
import torch

sys.path.insert(0, "/root/reference/src")
sys.modules["seaborn"] = types.ModuleType("seaborn")
import models as ref_models  # noqa: E402
import resolution_comparison as ref_rc  # noqa: E402


def main():
    d, out = sys.argv[1], sys.argv[2]
    torch.set_num_threads(os.cpu_count())
    sd = torch.load(os.path.join(d, "e2e_best_weights.pt"), weights_only=True)
    m = ref_models.UNet()
    m.load_state_dict(sd)
    m.eval()
    ours = np.load(os.path.join(d, "e2e_seed0_cascade.npz"))
    np.random.seed(0)
    data = ref_rc.solve_multi_resolution(40, [80, 160, 320, 640])
    rec = {"what": "trained-model cascade: HIP (GPU) vs the reference's code (CPU fp32), seed-0 field",
           "levels": {}}
    for r in (80, 160, 320, 640):
        ref = ref_rc.ml_multi_level_upscale(m, data, r, "cpu")
        got = ours[f"ml{r}"].astype(np.float64)
        e = got - ref
        rec["levels"][str(r)] = {"rmse_hip_vs_reference": float(np.sqrt(np.mean(e ** 2))),
                                 "max_abs": float(np.abs(e).max()),
                                 "field_rms": float(np.sqrt(np.mean(ref ** 2))),
                                 "reference_mae_vs_gt": float(np.mean(np.abs(ref - data["u"][r]))),
                                 "hip_mae_vs_gt": float(np.mean(np.abs(got - data["u"][r])))}
    rec["north_star_rmse_bar"] = 1e-5
    rec["pass"] = all(v["rmse_hip_vs_reference"] <= 1e-5 for v in rec["levels"].values())
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
