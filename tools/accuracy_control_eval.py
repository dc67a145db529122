"""Config #5 accuracy control, evaluation (build container, CPU): runs trained checkpoints through the
REFERENCE's own resolution comparison -- solve_multi_resolution(40, [80, 160, 320, 640]) and
ml_multi_level_upscale (src/resolution_comparison.py:13-229) plus the bilinear / bicubic multi-level and direct
baselines (src/resolution_comparison_enhanced.py:19-65, 355-408) -- on test fields np.random.seed(0 .. S-1), and
reports per model the mean MAE / RMSE per resolution and the ML / best-interpolation MAE ratio.

    PYTHONDONTWRITEBYTECODE=1 python tools/accuracy_control_eval.py OUT.json NAME=weights.pt [NAME=weights.pt ...]
(a weights file is a state dict, or a checkpoint dict holding 'model_state_dict')
"""
import json
import os
import sys
import types

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, "/root/reference/src")
sys.modules["seaborn"] = types.ModuleType("seaborn")
import models as ref_models  # noqa: E402  (reference)
import resolution_comparison as ref_rc  # noqa: E402
import resolution_comparison_enhanced as ref_rce  # noqa: E402

RES = (80, 160, 320, 640)


def load(path):
    sd = torch.load(path, map_location="cpu", weights_only=True)
    sd = sd.get("model_state_dict", sd)
    m = ref_models.UNet()
    m.load_state_dict(sd)
    return m.eval()


def interp(u40, res, mode):
    return F.interpolate(torch.from_numpy(u40).float()[None, None], size=(res, res), mode=mode,
                         align_corners=True).squeeze().numpy()


def main():
    out = sys.argv[1]
    models = {kv.split("=", 1)[0]: load(kv.split("=", 1)[1]) for kv in sys.argv[2:]}
    seeds = int(os.environ.get("ACC_SEEDS", "5"))
    torch.set_num_threads(os.cpu_count())
    per = []
    for seed in range(seeds):
        np.random.seed(seed)
        data = ref_rc.solve_multi_resolution(40, list(RES))
        rec = {"seed": seed, "k1": data["k1"], "k2": data["k2"], "mae": {}, "rmse": {}}
        sols = {}
        for r in RES:
            gt = data["u"][r]
            cand = {"bilinear_multi": ref_rce.bilinear_multi_level_upscale(data, r),
                    "cubic_multi": ref_rce.cubic_multi_level_upscale(data, r),
                    "bilinear_direct": interp(data["u"][40], r, "bilinear"),
                    "cubic_direct": interp(data["u"][40], r, "bicubic")}
            with torch.no_grad():
                for name, m in models.items():
                    cand[name] = ref_rc.ml_multi_level_upscale(m, data, r, "cpu")
            for k, v in cand.items():
                rec["mae"].setdefault(k, {})[str(r)] = float(np.mean(np.abs(v - gt)))
                rec["rmse"].setdefault(k, {})[str(r)] = float(np.sqrt(np.mean((v - gt) ** 2)))
        per.append(rec)
        print(json.dumps({"seed": seed, "mae640": {k: v["640"] for k, v in rec["mae"].items()}}), flush=True)
    summ = {}
    for k in per[0]["mae"]:
        summ[k] = {str(r): {"mae": float(np.mean([p["mae"][k][str(r)] for p in per])),
                            "rmse": float(np.mean([p["rmse"][k][str(r)] for p in per]))} for r in RES}
    interp_names = [k for k in summ if k not in models]
    ratio = {name: {str(r): summ[name][str(r)]["mae"] / min(summ[i][str(r)]["mae"] for i in interp_names)
                    for r in RES} for name in models}
    rec = {"what": "trained checkpoints through the reference's own resolution comparison (CPU fp32), test fields "
                   f"np.random.seed(0..{seeds - 1})", "mean_over_seeds": summ,
           "ml_over_best_interp_mae": ratio, "per_seed": per}
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps({"ml_over_best_interp_mae": ratio}, indent=1))


if __name__ == "__main__":
    main()
