"""Config #5 accuracy control, HIP side (verdict r5 item 4): the same dataset as tools/accuracy_control_ref.py
(np.random.seed(42), 1000 standard + 1000 subdomain samples; generated here by the batched HIP CG, which draws
the reference's sequence -- tests/test_gpu_poisson.py::test_generate_dataset_matches_reference), saved as the
reference's .npz and trained by train_enhanced.main(["--data", ...]) exactly as the reference's main (seed 42,
stratified split, batch 32, AdamW, ReduceLROnPlateau, clip 1.0, early stopping 20, --epochs cap).  Writes the
best weights (model_state_dict, fp32) for tools/accuracy_control_eval.py.

    python tools/accuracy_control_gpu.py --out gpurun_out/acc [--epochs 500]
"""
import argparse
import glob
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/acc")
    ap.add_argument("--epochs", type=int, default=500)
    ap.add_argument("--torch-seeds", type=int, nargs="*", default=[42],
                    help="train once per torch seed (model init + batch order; the data split keeps np seed 42): "
                         "the run-to-run spread of the trained model")
    a = ap.parse_args()
    from superresolution_for_pdes_amd import train_enhanced as T
    os.makedirs(a.out, exist_ok=True)
    np.random.seed(42)
    t0 = time.perf_counter()
    data = T.generate_on_device(1000, 1000, keep_on_device=False)
    npz = "/tmp/srpde_acc_dataset.npz"
    np.savez(npz, **data)
    gen_s = time.perf_counter() - t0
    real_seed, real_cuda_seed = torch.manual_seed, torch.cuda.manual_seed
    for ts in a.torch_seeds:
        # main() seeds torch (and the device generator, which draws the device-side init) with 42: this run's seed
        torch.manual_seed = (lambda _s, ts=ts: real_seed(ts))
        torch.cuda.manual_seed = (lambda _s, ts=ts: real_cuda_seed(ts))
        t0 = time.perf_counter()
        try:
            hist = T.main(["--data", npz, "--epochs", str(a.epochs), "--results", f"/tmp/srpde_acc_runs_{ts}"])
        finally:
            torch.manual_seed, torch.cuda.manual_seed = real_seed, real_cuda_seed
        torch.cuda.synchronize()
        train_s = time.perf_counter() - t0
        best = sorted(glob.glob(f"/tmp/srpde_acc_runs_{ts}/*/best_model.pth"))[-1]
        sd = torch.load(best, map_location="cpu", weights_only=True)["model_state_dict"]
        tag = f"hip_e{a.epochs}" + ("" if ts == 42 else f"_s{ts}")
        torch.save({k: v.float() if v.is_floating_point() else v for k, v in sd.items()},
                   os.path.join(a.out, f"{tag}_best_weights.pt"))
        rec = {"what": "HIP train_enhanced.main on the seed-42 dataset", "torch_seed": ts, "epochs_cap": a.epochs,
               "epochs_run": len(hist["train_loss"]), "best_epoch": hist["best_epoch"],
               "best_val_loss": hist["best_val_loss"], "train_loss": hist["train_loss"], "val_loss": hist["val_loss"],
               "generate_s": round(gen_s, 2), "train_s": round(train_s, 1),
               "dataset_checksum": {k: float(np.asarray(v, dtype=np.float64).sum()) for k, v in data.items()}}
        json.dump(rec, open(os.path.join(a.out, f"{tag}_history.json"), "w"))
        print(json.dumps({k: v for k, v in rec.items() if k not in ("train_loss", "val_loss", "dataset_checksum")}),
              flush=True)


if __name__ == "__main__":
    main()
