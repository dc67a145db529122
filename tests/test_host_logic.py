"""CPU: host-side logic of the drop-in surface (no kernel launches)."""
import json
import os

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_state_dict_contract_matches_reference():
    from superresolution_for_pdes_amd.models import UNet
    keys = json.load(open(os.path.join(ROOT, "tests", "golden", "state_keys.json")))
    sd = UNet().state_dict()
    assert [[k, list(v.shape)] for k, v in sd.items()] == keys
    assert len(sd) == 132
    assert sum(p.numel() for p in UNet().parameters()) == 7834588


def test_oracle_spec_matches_reference_keys():
    from oracle.unet_ref import param_specs
    keys = json.load(open(os.path.join(ROOT, "tests", "golden", "state_keys.json")))
    assert [[n, list(s)] for n, s, _ in param_specs()] == keys


def test_flat_layout_is_backward_completion_order():
    from superresolution_for_pdes_amd import unet_exec as X
    from superresolution_for_pdes_amd.models import UNet
    m = UNet()
    lay = X.flat_layout(m)
    assert lay[0][0].startswith("final.") and lay[-1][0].startswith("enc1.")
    offs = [o for _, _, o, _ in lay]
    assert offs == sorted(offs) and lay[-1][2] + lay[-1][3] == 7834588
    ends = X._group_end_offsets(lay)
    seq = [ends[g] for g in X.FLAT_GROUPS]
    assert seq == sorted(seq)


def test_flatten_parameters_rehomes_views_cpu():
    from superresolution_for_pdes_amd.models import UNet
    m = UNet()
    before = {n: p.detach().clone() for n, p in m.named_parameters()}
    fp = m.flatten_parameters_()
    for n, p in m.named_parameters():
        assert torch.equal(p.detach(), before[n])
    for _, p, off, _ in m._flat_layout():
        assert p.data_ptr() == fp.data_ptr() + 4 * off
    sd = m.state_dict()
    m.load_state_dict(sd)  # in-place copies keep the views
    assert m.flatten_parameters_() is fp


def test_fused_adamw_flat_span_detection():
    from superresolution_for_pdes_amd.optim import _flat_span
    base = torch.zeros(10)
    a, b = base[0:4].view(2, 2), base[4:10]
    assert _flat_span([a, b]).numel() == 10
    assert _flat_span([b, a]) is None
    assert _flat_span([a, torch.zeros(6)]) is None


def test_shard_indices_distributed_sampler_semantics():
    from superresolution_for_pdes_amd.distributed import shard_indices
    n, world = 10, 4
    shards = [shard_indices(n, r, world, seed=5) for r in range(world)]
    assert all(len(s) == 3 for s in shards)
    allidx = torch.cat(shards)
    assert set(allidx.tolist()) == set(range(n))
    assert torch.equal(shard_indices(n, 1, world, 5), shards[1])
    assert not torch.equal(shard_indices(n, 1, world, 5, epoch=1), shards[1])


def test_stratified_split_follows_reference_rng_order():
    """train_enhanced.py:232-268: permutation, then the two shuffles, then two more."""
    from superresolution_for_pdes_amd.train_enhanced import stratified_split
    flags = np.array([False] * 7 + [True] * 5)
    data = {"u_fine": np.zeros((12, 2, 2)), "is_subdomain": flags}
    np.random.seed(42)
    tr, va = stratified_split(data, 0.2, True)
    np.random.seed(42)
    np.random.permutation(12)
    sub, std = np.where(flags)[0], np.where(~flags)[0]
    np.random.shuffle(sub)
    np.random.shuffle(std)
    tr2 = np.concatenate([std[1:], sub[1:]])
    va2 = np.concatenate([std[:1], sub[:1]])
    np.random.shuffle(tr2)
    np.random.shuffle(va2)
    assert np.array_equal(tr, tr2) and np.array_equal(va, va2)
    assert len(set(tr) | set(va)) == 12 and not set(tr) & set(va)


def test_reference_config_keys():
    from superresolution_for_pdes_amd.train_enhanced import default_config
    assert set(default_config()) == {"batch_size", "num_epochs", "learning_rate", "min_lr", "patience",
                                     "early_stopping_patience", "val_split", "grad_clip", "device", "num_workers",
                                     "pin_memory", "stratify_by_subdomain"}


def test_cpu_tensors_fail_loudly():
    """No CPU fallback: the HIP modules refuse host tensors."""
    import pytest
    from superresolution_for_pdes_amd.models import UNet, PDEDataset
    from superresolution_for_pdes_amd.functional import mse_loss
    with pytest.raises(RuntimeError):
        UNet().eval()(torch.zeros(1, 3, 40, 40))
    with pytest.raises(RuntimeError):
        mse_loss(torch.zeros(4), torch.zeros(4))
    with pytest.raises(RuntimeError):
        PDEDataset({"u_coarse": np.zeros((1, 20, 20)), "u_fine": np.zeros((1, 40, 40)),
                    "f_fine": np.zeros((1, 40, 40)), "theta_fine": np.ones((1, 40, 40))}, device="cpu")


def test_bench_refuses_world_size_mismatch():
    """bench.py exits non-zero, before any GPU call, when WORLD_SIZE disagrees with --gpus."""
    import subprocess
    import sys
    env = dict(os.environ, WORLD_SIZE="4", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--no-cpu-baseline"],
                       env=env, capture_output=True, text=True, timeout=120)
    assert p.returncode == 2 and "WORLD_SIZE=4" in p.stderr


def test_init_weights_matches_reference_seeded():
    """M10: torch.manual_seed(42); UNet().apply(init_weights) -- as train_enhanced.main does
    (:187-189, :303-304) -- builds the reference's initial tensors bit for bit (init_fixture: the
    reference's own run, models.py:209-222; same module registration order, same RNG draws)."""
    from superresolution_for_pdes_amd.models import UNet, init_weights
    z = np.load(os.path.join(ROOT, "tests", "golden", "init_fixture.npz"))
    torch.manual_seed(42)
    m = UNet()
    m.apply(init_weights)
    sd = m.state_dict()
    keys = {k.split(":", 1)[1] for k in z.files}
    assert keys == set(sd)
    for k, v in sd.items():
        if not v.is_floating_point():
            assert np.array_equal(v.numpy(), z[f"int:{k}"]), k
            continue
        f = v.detach().reshape(-1).double()
        assert float(f.norm()) == float(z[f"norm:{k}"]), k
        assert float(f.sum()) == float(z[f"sum:{k}"]), k
        assert np.array_equal(f[:: max(1, f.numel() // 64)][:64].numpy(), z[f"sample:{k}"]), k
