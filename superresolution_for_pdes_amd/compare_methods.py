"""``load_model`` of reference src/compare_methods.py:11-17 (the checkpoint boundary).

Reference checkpoints (``best_model.pth`` / ``final_model.pth``, train_enhanced.py:117-125,
:341-351) hold ``model_state_dict`` with the reference's 132 keys, which the HIP ``UNet``
shares, so they load unchanged.  Loaded with ``weights_only=True`` (nothing executed).
"""
from __future__ import annotations

from pathlib import Path

import torch

from .models import UNet


def load_model(checkpoint_path: Path, device: str = "cuda") -> UNet:
    model = UNet().to(device)
    checkpoint = torch.load(checkpoint_path, map_location=device, weights_only=True)
    model.load_state_dict(checkpoint["model_state_dict"])
    model.eval()
    return model
