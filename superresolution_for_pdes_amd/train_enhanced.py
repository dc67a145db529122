"""Drop-in for reference ``src/train_enhanced.py`` on MI355X.

``train_model`` keeps the reference signature and history dict (train_enhanced.py:15-139):
per batch zero_grad -> forward -> criterion -> backward -> clip_grad_norm_(grad_clip) ->
optimizer.step(); validation under no_grad; ReduceLROnPlateau on the val loss; best
checkpoint on improvement; early stopping.  Differences that do not change results:

* the batch loss is accumulated ON DEVICE and read once per epoch (the reference's
  per-batch ``loss.item()`` host sync, :77, is gone);
* with ``FusedAdamW`` the clip + update is one fused HIP pass (same math);
* batches are gathered by index on the device (``DeviceBatchLoader``) -- the reference's
  DataLoader workers (:286-300) cannot touch device tensors anyway;
* ``main`` accepts overrides (``--epochs``, ``--batch-size``, ``--data``, ``--generate``
  for on-device data generation, config #3) and runs data-parallel over RCCL when
  launched with torchrun (one process per GPU, distributed.DataParallel): the generated
  dataset's solves are sharded over the ranks and all-gathered, the batch size is per rank
  (global batch = world x batch), and validation deals the single-process batches to the
  ranks so the reduced val loss (which drives the scheduler, checkpoints and early stopping)
  equals the single-process value.
"""
from __future__ import annotations

import argparse
import json
import os
from datetime import datetime
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist
import torch.nn as nn
import torch.optim as optim

from .functional import MSELoss
from .models import PDEDataset, UNet, init_weights
from .optim import FusedAdamW


class ScalarWriter:
    """TensorBoard-compatible add_scalar/close; uses torch.utils.tensorboard when installed,
    else appends JSON lines (same tags: 'Loss/train', 'Loss/val', 'Learning_rate')."""

    def __init__(self, log_dir):
        self.tb = None
        try:
            from torch.utils.tensorboard import SummaryWriter
            self.tb = SummaryWriter(log_dir=log_dir)
        except Exception:  # tensorboard is optional (absent in this image)
            Path(log_dir).mkdir(parents=True, exist_ok=True)
            self.f = open(Path(log_dir) / "scalars.jsonl", "a")

    def add_scalar(self, tag, value, step):
        if self.tb is not None:
            self.tb.add_scalar(tag, value, step)
        else:
            self.f.write(json.dumps({"tag": tag, "value": float(value), "step": int(step)}) + "\n")
            self.f.flush()

    def close(self):
        if self.tb is not None:
            self.tb.close()
        else:
            self.f.close()


class DeviceBatchLoader:
    """Index-gathered batches from a device-resident PDEDataset (DataLoader replacement).

    shuffle: a seeded permutation per epoch; with world > 1 each rank takes a disjoint
    strided shard of it (DistributedSampler semantics: ``batch_size`` is per rank, the global
    batch is world x batch_size, as under torch DDP).  ``shard_batches`` (evaluation): the
    single-process batches themselves are dealt round-robin to the ranks, unpadded, so the
    all-reduced (sum of batch losses, batch count) gives exactly the single-process mean."""

    def __init__(self, dataset, batch_size, shuffle=False, seed=0, rank=0, world=1, drop_last=False,
                 shard_batches=False):
        self.ds, self.bs, self.shuffle = dataset, batch_size, shuffle
        self.seed, self.rank, self.world, self.drop_last = seed, rank, world, drop_last
        self.shard_batches = shard_batches
        self.epoch = 0

    def _indices(self):
        from .distributed import shard_indices
        n = len(self.ds)
        if self.world > 1 and not self.shard_batches:
            return shard_indices(n, self.rank, self.world, self.seed, self.epoch, self.shuffle)
        if self.shuffle:
            g = torch.Generator().manual_seed(self.seed + self.epoch)
            return torch.randperm(n, generator=g)
        return torch.arange(n)

    def _batches(self, idx):
        out = [idx[s:s + self.bs] for s in range(0, len(idx), self.bs)]
        if self.drop_last and out and len(out[-1]) < self.bs:
            out = out[:-1]
        if self.shard_batches and self.world > 1:
            out = out[self.rank::self.world]
        return out

    def __len__(self):
        return len(self._batches(self._indices()))

    def __iter__(self):
        idx = self._indices().to(self.ds.inputs.device)
        self.epoch += 1
        for b in self._batches(idx):
            yield self.ds.batch(b)


def _is_main():
    return not dist.is_initialized() or dist.get_rank() == 0


def _global_mean(total, count, device):
    """(sum of batch losses, number of batches) summed over ranks -> the mean batch loss, the
    reference's ``loss_sum / len(loader)`` (train_enhanced.py:79, :92) over all ranks' batches."""
    t = torch.stack([total.to(torch.float64), torch.tensor(float(count), dtype=torch.float64, device=device)])
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t)
    return float(t[0] / torch.clamp(t[1], min=1.0))


def train_model(model: nn.Module, train_loader, val_loader, criterion: nn.Module, optimizer: optim.Optimizer,
                scheduler, num_epochs: int, device: str, save_dir: Path, writer, grad_clip: float = 1.0,
                early_stopping_patience: int = 20) -> dict:
    """Train with per-epoch validation, checkpointing and early stopping (train_enhanced.py:15-139)."""
    history = {"train_loss": [], "val_loss": [], "best_val_loss": float("inf"), "best_epoch": 0, "num_epochs": 0}
    no_improvement_count = 0
    save_dir = Path(save_dir)
    fused = isinstance(optimizer, FusedAdamW)
    module = model.module if hasattr(model, "module") else model
    for epoch in range(num_epochs):
        model.train()
        acc = torch.zeros((), dtype=torch.float64, device=device)
        nb = 0
        for inputs, targets in train_loader:
            inputs, targets = inputs.to(device), targets.to(device)
            optimizer.zero_grad()
            outputs = model(inputs)
            loss = criterion(outputs, targets)
            loss.backward()
            if fused:
                optimizer.step(max_grad_norm=grad_clip)
            else:
                torch.nn.utils.clip_grad_norm_(module.parameters(), grad_clip)
                optimizer.step()
            acc += loss.detach()
            nb += 1
        train_loss = _global_mean(acc, nb, device)

        # under data parallelism each rank's last training forward updated its BN running
        # statistics with its own shard: validate every rank with rank 0's buffers (the state
        # best_model.pth saves), so the reduced val loss is that model's single-process loss
        if hasattr(model, "sync_buffers"):
            model.sync_buffers()
        model.eval()
        vacc = torch.zeros((), dtype=torch.float64, device=device)
        vb = 0
        with torch.no_grad():
            for inputs, targets in val_loader:
                inputs, targets = inputs.to(device), targets.to(device)
                vacc += criterion(model(inputs), targets).detach()
                vb += 1
        val_loss = _global_mean(vacc, vb, device)

        scheduler.step(val_loss)
        current_lr = optimizer.param_groups[0]["lr"]
        if writer is not None:
            writer.add_scalar("Loss/train", train_loss, epoch)
            writer.add_scalar("Loss/val", val_loss, epoch)
            writer.add_scalar("Learning_rate", current_lr, epoch)
        history["train_loss"].append(train_loss)
        history["val_loss"].append(val_loss)
        if _is_main():
            print(f"Epoch {epoch + 1}/{num_epochs}:\nTrain Loss: {train_loss:.6f}\nVal Loss: {val_loss:.6f}\n"
                  f"Learning Rate: {current_lr:.6f}")
        if val_loss < history["best_val_loss"]:
            history["best_val_loss"] = val_loss
            history["best_epoch"] = epoch
            no_improvement_count = 0
            if _is_main():
                torch.save({"epoch": epoch, "model_state_dict": module.state_dict(),
                            "optimizer_state_dict": optimizer.state_dict(),
                            "scheduler_state_dict": scheduler.state_dict(),
                            "train_loss": train_loss, "val_loss": val_loss}, save_dir / "best_model.pth")
                print(f"Saved new best model with val_loss: {val_loss:.6f}")
        else:
            no_improvement_count += 1
            if _is_main():
                print(f"No improvement for {no_improvement_count} epochs (best: {history['best_val_loss']:.6f} "
                      f"at epoch {history['best_epoch'] + 1})")
        if no_improvement_count >= early_stopping_patience:
            if _is_main():
                print(f"Early stopping triggered after {epoch + 1} epochs")
            break
    history["num_epochs"] = len(history["train_loss"])
    return history


def plot_losses(history: dict, save_dir: Path):
    """training_history.png (train_enhanced.py:141-183)."""
    try:
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
    except Exception:
        return
    plt.figure(figsize=(12, 7))
    epochs = range(1, len(history["train_loss"]) + 1)
    plt.plot(epochs, history["train_loss"], "b-", label="Training Loss")
    plt.plot(epochs, history["val_loss"], "r-", label="Validation Loss")
    be = history["best_epoch"] + 1
    plt.plot(be, history["best_val_loss"], "go", markersize=10,
             label=f"Best Model (Epoch {be}, Loss: {history['best_val_loss']:.6f})")
    plt.xlabel("Epoch")
    plt.ylabel("Loss")
    plt.title("Training and Validation Loss")
    plt.legend()
    plt.grid(True, alpha=0.3)
    plt.tight_layout()
    plt.savefig(Path(save_dir) / "training_history.png", dpi=150)
    plt.close()


def stratified_split(data, val_split=0.2, stratify=True):
    """Index split with the reference's np.random call order (train_enhanced.py:232-268)."""
    n_samples = len(data["u_fine"])
    indices = np.random.permutation(n_samples)
    val_size = int(n_samples * val_split)
    if stratify and "is_subdomain" in data:
        sub = np.where(data["is_subdomain"])[0]
        std = np.where(~data["is_subdomain"])[0]
        np.random.shuffle(sub)
        np.random.shuffle(std)
        vs, vt = int(len(sub) * val_split), int(len(std) * val_split)
        train_idx = np.concatenate([std[vt:], sub[vs:]])
        val_idx = np.concatenate([std[:vt], sub[:vs]])
        np.random.shuffle(train_idx)
        np.random.shuffle(val_idx)
    else:
        train_idx, val_idx = indices[val_size:], indices[:val_size]
    return train_idx, val_idx


def default_config():
    """The reference's config dict (train_enhanced.py:192-205)."""
    return {
        "batch_size": 32, "num_epochs": 500, "learning_rate": 2e-4, "min_lr": 1e-6, "patience": 10,
        "early_stopping_patience": 20, "val_split": 0.2, "grad_clip": 1.0,
        "device": "cuda" if torch.cuda.is_available() else "cpu",
        "num_workers": 4, "pin_memory": True, "stratify_by_subdomain": True,
    }


def generate_on_device(n_standard=1000, n_subdomain=1000, keep_on_device=True, shard=None):
    """Config #3: the enhanced_data_generation.py __main__ dataset built by the HIP solver.
    The fields stay device tensors from the batched CG to PDEDataset; under
    torchrun the solves are sharded over the ranks and all-gathered (8(e)), the draws global."""
    from .enhanced_data_generation import EnhancedPoissonSolver
    s = EnhancedPoissonSolver(20, 40, 80)
    d1 = s.generate_dataset(n_samples=n_standard, k_range=(0.5, 5.0), keep_on_device=keep_on_device, shard=shard)
    d2 = s.generate_subdomain_dataset(n_samples=n_subdomain, k_range=(0.5, 12.0), keep_on_device=keep_on_device,
                                      shard=shard)
    return s.combine_datasets(d1, d2)


def _per_sample(v):
    return (v.ndim if hasattr(v, "ndim") else np.ndim(v)) > 0


def select(data: dict, idx) -> dict:
    """Rows ``idx`` of every per-sample field (device tensors indexed on the device)."""
    out = {}
    for k, v in data.items():
        if not _per_sample(v):
            continue
        out[k] = v[torch.as_tensor(idx, device=v.device)] if isinstance(v, torch.Tensor) else v[idx]
    return out


def main(argv=None):
    ap = argparse.ArgumentParser(description="MI355X U-Net training (reference train_enhanced.main)")
    ap.add_argument("--data", default="data/pde_dataset.npz")
    ap.add_argument("--generate", type=int, nargs=2, metavar=("N_STD", "N_SUB"), default=None,
                    help="generate the dataset on device instead of loading --data")
    ap.add_argument("--epochs", type=int, default=None)
    ap.add_argument("--batch-size", type=int, default=None,
                    help="per-rank batch (under torchrun the global batch is world x batch-size, as torch DDP)")
    ap.add_argument("--results", default="results")
    args = ap.parse_args(argv)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1 and not dist.is_initialized():
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    rank = dist.get_rank() if dist.is_initialized() else 0

    torch.manual_seed(42)
    np.random.seed(42)
    torch.cuda.manual_seed(42)
    config = default_config()
    if args.epochs is not None:
        config["num_epochs"] = args.epochs
    if args.batch_size is not None:
        config["batch_size"] = args.batch_size
    device = f"cuda:{torch.cuda.current_device()}" if torch.cuda.is_available() else "cpu"

    save_dir = Path(args.results) / f"enhanced_run_{datetime.now().strftime('%Y%m%d_%H%M%S')}"
    if rank == 0:
        save_dir.mkdir(parents=True, exist_ok=True)
        with open(save_dir / "config.json", "w") as f:
            json.dump(config, f, indent=4)
    writer = ScalarWriter(str(save_dir / "tensorboard")) if rank == 0 else None

    if args.generate is not None:
        data = generate_on_device(*args.generate)
    else:
        data = dict(np.load(args.data))
    train_idx, val_idx = stratified_split(data, config["val_split"], config["stratify_by_subdomain"])
    train_ds = PDEDataset(select(data, train_idx), device=device)
    val_ds = PDEDataset(select(data, val_idx), device=device)
    train_loader = DeviceBatchLoader(train_ds, config["batch_size"], shuffle=True, seed=42, rank=rank, world=world)
    val_loader = DeviceBatchLoader(val_ds, config["batch_size"], shuffle=False, rank=rank, world=world,
                                   shard_batches=True)

    model = UNet().to(device)
    model.apply(init_weights)
    net = model
    if world > 1:
        from .distributed import DataParallel
        net = DataParallel(model)
    criterion = MSELoss()
    optimizer = FusedAdamW(model.parameters(), lr=config["learning_rate"], weight_decay=1e-4)
    scheduler = optim.lr_scheduler.ReduceLROnPlateau(optimizer, mode="min", factor=0.5, patience=config["patience"],
                                                     min_lr=config["min_lr"])
    history = train_model(net, train_loader, val_loader, criterion, optimizer, scheduler, config["num_epochs"],
                          device, save_dir, writer, config["grad_clip"], config["early_stopping_patience"])
    if rank == 0:
        plot_losses(history, save_dir)
        torch.save({"epoch": len(history["train_loss"]) - 1, "model_state_dict": model.state_dict(),
                    "optimizer_state_dict": optimizer.state_dict(), "scheduler_state_dict": scheduler.state_dict(),
                    "train_loss": history["train_loss"][-1], "val_loss": history["val_loss"][-1],
                    "best_val_loss": history["best_val_loss"], "best_epoch": history["best_epoch"]},
                   save_dir / "final_model.pth")
        print(f"\nTraining Summary:\nTotal epochs: {len(history['train_loss'])}\n"
              f"Best validation loss: {history['best_val_loss']:.6f} (epoch {history['best_epoch'] + 1})")
        writer.close()
    return history


if __name__ == "__main__":
    main()
