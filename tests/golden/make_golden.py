"""Generate the golden fixtures by running the REAL reference (read-only import).

Run in the build container only (``/root/reference`` does not exist on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

Writes small ``.npz`` / ``.json`` files next to this script.  Everything written is
data (inputs and the reference's outputs); no reference source is copied.  The
reference is imported from ``/root/reference/src`` with two in-process stubs
(``torch.utils.tensorboard`` and ``seaborn``, both absent here and only used for
logging/plots), as SURVEY.md 8(c) describes.

Fixtures:
  state_keys.json      reference UNet().state_dict() names + shapes (132 entries)
  unet_fixture.npz     fwd eval/train fp32 + fp64, running stats, MSE grads (norms and
                       samples), one clip+AdamW step (param samples)  [B=4]
  poisson_fixture.npz  spsolve at n=20/40/80/160 (theta=1 and theta~U(0.5,2)), n=640 stats
  datagen_fixture.npz  generate_dataset / generate_subdomain_dataset / combine_datasets
                       with seeded np.random, PDEDataset stats and items
  cascade_fixture.npz  solve_multi_resolution(40,[80,160]) + ml_multi_level_upscale to 160
"""
from __future__ import annotations

import json
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, HERE)
REF = "/root/reference/src"
sys.path.insert(0, REF)

# --- stubs for plot/log-only dependencies absent from this container -------------
tb = types.ModuleType("torch.utils.tensorboard")


class _Writer:
    def __init__(self, *a, **k):
        pass

    def add_scalar(self, *a, **k):
        pass

    def close(self):
        pass


tb.SummaryWriter = _Writer
sys.modules["torch.utils.tensorboard"] = tb
sys.modules["seaborn"] = types.ModuleType("seaborn")

import models as ref_models  # noqa: E402  (reference)
import data_generation as ref_dg  # noqa: E402
import enhanced_data_generation as ref_edg  # noqa: E402
import resolution_comparison as ref_rc  # noqa: E402

from state import fixture_state_torch, fixture_inputs, sample_indices  # noqa: E402
from oracle.unet_ref import trainable_names  # noqa: E402


def ref_model(dtype):
    m = ref_models.UNet()
    st = fixture_state_torch(dtype=dtype)
    m.load_state_dict(st)
    return m.to(dtype)


def unet_fixture():
    torch.set_num_threads(8)
    x, t = fixture_inputs(4)
    out = {"x": x, "t": t}
    names = trainable_names()
    for tag, dt in (("32", torch.float32), ("64", torch.float64)):
        xx = torch.from_numpy(x).to(dt)
        tt = torch.from_numpy(t).to(dt)
        m = ref_model(dt).eval()
        with torch.no_grad():
            out[f"out_eval{tag}"] = m(xx).numpy()
        m = ref_model(dt).train()
        y = m(xx)
        loss = torch.nn.MSELoss()(y, tt)
        loss.backward()
        out[f"out_train{tag}"] = y.detach().numpy()
        out[f"loss{tag}"] = np.array(loss.item())
        sd = m.state_dict()
        for k, v in sd.items():
            if k.endswith("running_mean") or k.endswith("running_var"):
                out[f"rs{tag}:{k}"] = v.numpy()
        params = dict(m.named_parameters())
        gn = []
        for i, n in enumerate(names):
            g = params[n].grad.detach().reshape(-1)
            gn.append(float(torch.linalg.vector_norm(g.double())))
            idx = sample_indices(g.numel(), 1000 + i)
            out[f"gidx:{n}"] = idx
            out[f"gval{tag}:{n}"] = g[idx].numpy()
        out[f"gnorm{tag}"] = np.array(gn)
        if tag == "32":
            # one clip + AdamW step exactly as train_enhanced.py:74-75, 308
            opt = torch.optim.AdamW(m.parameters(), lr=2e-4, weight_decay=1e-4)
            tot = torch.nn.utils.clip_grad_norm_(m.parameters(), 1.0)
            out["clip_total32"] = np.array(float(tot))
            opt.step()
            for i, n in enumerate(names):
                p = params[n].detach().reshape(-1)
                out[f"pval{tag}:{n}"] = p[out[f"gidx:{n}"]].numpy()
    np.savez_compressed(os.path.join(HERE, "unet_fixture.npz"), **out)
    keys = [[k, list(v.shape)] for k, v in ref_models.UNet().state_dict().items()]
    with open(os.path.join(HERE, "state_keys.json"), "w") as f:
        json.dump(keys, f, indent=0)


def poisson_fixture():
    out = {}
    rng = np.random.default_rng(11)
    for n in (20, 40, 80, 160):
        solver = ref_dg.PoissonSolver(n_coarse=n // 2, n_fine=n)
        k1, k2 = 1.3 + n / 100.0, 3.7 - n / 200.0
        f = solver.generate_forcing_term(k1, k2, "fine")
        th1 = np.ones((n, n))
        thv = rng.uniform(0.5, 2.0, (n, n))
        out[f"f{n}"] = f
        out[f"k{n}"] = np.array([k1, k2])
        out[f"thv{n}"] = thv
        out[f"u1_{n}"] = solver.solve_poisson(f, th1, "fine")
        out[f"uv_{n}"] = solver.solve_poisson(f, thv, "fine")
    # 640: too big to store whole; keep its inputs' seed-free definition + stats/slices
    n = 640
    solver = ref_dg.PoissonSolver(n_coarse=n // 2, n_fine=n)
    f = solver.generate_forcing_term(10.25, 10.75, "fine")
    thv = np.random.default_rng(640).uniform(0.5, 2.0, (n, n))
    u = solver.solve_poisson(f, thv, "fine")
    out["u640_norm"] = np.array(np.linalg.norm(u))
    out["u640_row320"] = u[320].copy()
    out["u640_col100"] = u[:, 100].copy()
    out["u640_sum"] = np.array(u.sum())
    np.savez_compressed(os.path.join(HERE, "poisson_fixture.npz"), **out)


def datagen_fixture():
    out = {}
    s = ref_edg.EnhancedPoissonSolver(20, 40, 80)
    np.random.seed(123)
    d1 = s.generate_dataset(n_samples=3, k_range=(0.5, 5.0))
    np.random.seed(7)
    d2 = s.generate_subdomain_dataset(n_samples=3, k_range=(0.5, 12.0))
    comb = s.combine_datasets(dict(d1), d2)
    for k, v in d1.items():
        out[f"std:{k}"] = v
    for k, v in d2.items():
        out[f"sub:{k}"] = v
    for k, v in comb.items():
        out[f"comb:{k}"] = v
    ds = ref_models.PDEDataset(comb, device="cpu")
    out["ds_u_mean"] = np.array(float(ds.u_mean))
    out["ds_u_std"] = np.array(float(ds.u_std))
    out["ds_f_mean"] = np.array(float(ds.f_mean))
    out["ds_f_std"] = np.array(float(ds.f_std))
    out["ds_theta_const"] = np.array(bool(ds.theta_is_constant))
    xs, ys = zip(*[ds[i] for i in range(len(ds))])
    out["ds_x"] = torch.stack(xs).numpy()
    out["ds_y"] = torch.stack(ys).numpy()
    # a variable-theta dataset exercises the theta-normalisation branch (models.py:169-170)
    varc = dict(comb)
    varc["theta_fine"] = np.random.default_rng(5).uniform(0.5, 2.0, comb["theta_fine"].shape)
    dsv = ref_models.PDEDataset(varc, device="cpu")
    out["dsv_theta_fine"] = varc["theta_fine"]
    xs, _ = zip(*[dsv[i] for i in range(len(dsv))])
    out["dsv_x"] = torch.stack(xs).numpy()
    np.savez_compressed(os.path.join(HERE, "datagen_fixture.npz"), **out)


def cascade_fixture():
    np.random.seed(0)
    data = ref_rc.solve_multi_resolution(40, [80, 160])
    m = ref_model(torch.float32).eval()
    out = {"k1": np.array(data["k1"]), "k2": np.array(data["k2"])}
    for r in (40, 80, 160):
        out[f"f{r}"] = data["f"][r]
        out[f"theta{r}"] = data["theta"][r]
        out[f"u{r}"] = data["u"][r]
    for tgt in (80, 160):
        out[f"ml{tgt}"] = ref_rc.ml_multi_level_upscale(m, data, tgt, "cpu")
    np.savez_compressed(os.path.join(HERE, "cascade_fixture.npz"), **out)


if __name__ == "__main__":
    unet_fixture()
    poisson_fixture()
    datagen_fixture()
    cascade_fixture()
    for f in sorted(os.listdir(HERE)):
        print(f, os.path.getsize(os.path.join(HERE, f)))
