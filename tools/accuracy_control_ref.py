"""Config #5 accuracy control, reference side (build container only, CPU; verdict r5 item 4).

Generates the reference's training set with the REFERENCE's own generators (np.random.seed(42), then
1000 standard samples with k ~ U(0.5, 5) and 1000 subdomain samples with k ~ U(0.5, 12), as
`train_enhanced.main(["--generate", "1000", "1000"])` draws them on the device), saves it as the
reference's 9-key `.npz`, and trains the REFERENCE's own `train_model` (src/train_enhanced.py:15-139) on it
on the CPU with the reference's config (batch 32, AdamW 2e-4 / 1e-4, ReduceLROnPlateau(0.5, 10, 1e-6),
clip 1.0, early stopping 20, `--epochs` cap, 500 in the reference's config.json), after the same seeding and
stratified split as its `main` (train_enhanced.py:187-189, 232-268).  The reference is imported read-only
with the SURVEY 8(c) stubs (tensorboard, seaborn); DataLoader workers are 0 (no fork; the batches are the
same).  The HIP side trains on the same `.npz` (tools/accuracy_control_gpu.py); tools/accuracy_control_eval.py
runs both checkpoints through the reference's own resolution comparison.

    PYTHONDONTWRITEBYTECODE=1 python tools/accuracy_control_ref.py --out /tmp/acc [--epochs 500]
"""
import argparse
import json
import os
import sys
import time
import types

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, "/root/reference/src")
tb = types.ModuleType("torch.utils.tensorboard")


class _Writer:
    def __init__(self, *a, **k):
        self.scalars = []

    def add_scalar(self, tag, v, step=None):
        self.scalars.append((tag, float(v), step))

    def close(self):
        pass


tb.SummaryWriter = _Writer
sys.modules["torch.utils.tensorboard"] = tb
sys.modules["seaborn"] = types.ModuleType("seaborn")
import enhanced_data_generation as ref_edg  # noqa: E402  (reference)
import models as ref_models  # noqa: E402
import train_enhanced as ref_te  # noqa: E402

from superresolution_for_pdes_amd.train_enhanced import stratified_split  # noqa: E402  (pure numpy index split)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="/tmp/acc")
    ap.add_argument("--epochs", type=int, default=500)
    ap.add_argument("--n", type=int, nargs=2, default=(1000, 1000))
    args = ap.parse_args()
    os.makedirs(args.out, exist_ok=True)
    torch.set_num_threads(os.cpu_count())
    npz = os.path.join(args.out, "pde_dataset.npz")
    if not os.path.exists(npz):
        t0 = time.perf_counter()
        np.random.seed(42)
        s = ref_edg.EnhancedPoissonSolver(n_coarse=20, n_fine=40, n_superfine=80)
        d1 = s.generate_dataset(n_samples=args.n[0], k_range=(0.5, 5.0))
        d2 = s.generate_subdomain_dataset(n_samples=args.n[1], k_range=(0.5, 12.0))
        data = s.combine_datasets(d1, d2)
        np.savez(npz, **data)
        print(f"dataset {sorted(data)} in {time.perf_counter() - t0:.1f} s", flush=True)
    data = dict(np.load(npz))

    # train_enhanced.main's order: seeds, split, datasets, loaders, model + init, loss, optimizer, scheduler
    torch.manual_seed(42)
    np.random.seed(42)
    tr, va = stratified_split(data, 0.2, True)
    train_ds = ref_models.PDEDataset({k: v[tr] for k, v in data.items()}, device="cpu")
    val_ds = ref_models.PDEDataset({k: v[va] for k, v in data.items()}, device="cpu")
    train_loader = torch.utils.data.DataLoader(train_ds, batch_size=32, shuffle=True, num_workers=0)
    val_loader = torch.utils.data.DataLoader(val_ds, batch_size=32, shuffle=False, num_workers=0)
    model = ref_models.UNet()
    model.apply(ref_models.init_weights)
    crit = torch.nn.MSELoss()
    opt = torch.optim.AdamW(model.parameters(), lr=2e-4, weight_decay=1e-4)
    sched = torch.optim.lr_scheduler.ReduceLROnPlateau(opt, mode="min", factor=0.5, patience=10, min_lr=1e-6)
    save = os.path.join(args.out, f"ref_e{args.epochs}")
    os.makedirs(save, exist_ok=True)
    writer = _Writer()
    t0 = time.perf_counter()
    from pathlib import Path
    hist = ref_te.train_model(model=model, train_loader=train_loader, val_loader=val_loader, criterion=crit,
                              optimizer=opt, scheduler=sched, num_epochs=args.epochs, device="cpu",
                              save_dir=Path(save), writer=writer, grad_clip=1.0, early_stopping_patience=20)
    rec = {"what": "reference train_model on CPU, reference config", "epochs_cap": args.epochs,
           "epochs_run": len(hist["train_loss"]), "best_epoch": hist["best_epoch"],
           "best_val_loss": hist["best_val_loss"], "train_loss": hist["train_loss"], "val_loss": hist["val_loss"],
           "wall_s": round(time.perf_counter() - t0, 1), "threads": torch.get_num_threads()}
    json.dump(rec, open(os.path.join(save, "history.json"), "w"))
    print(json.dumps({k: v for k, v in rec.items() if k not in ("train_loss", "val_loss")}), flush=True)


if __name__ == "__main__":
    main()
