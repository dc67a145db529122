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
  unet_b1024_fixture.npz  the bench configuration (#2): B=1024 train-mode forward + MSE backward
                       + clip + AdamW in fp64 and fp32 (output samples and per-sample sums, all
                       16 BNs' running stats, per-parameter gradient norms and samples, one
                       optimizer step).  The fp64 run wraps the reference's blocks in
                       torch.utils.checkpoint (same ops, recomputed in backward) to fit in host
                       memory; running stats are read before the recompute touches them.
  cascade640_fixture.npz  solve_multi_resolution(40,[80..640]) + ml_multi_level_upscale to
                       320 and 640, plus the bilinear / bicubic multi-level and direct baselines
                       (resolution_comparison_enhanced.py:19-65, :355-408) and their metrics
  init_fixture.npz     torch.manual_seed(42); UNet().apply(init_weights) as train_enhanced.main
                       does (:187-189, :303-304): per-parameter norms, sums and strided samples
  report_fixture.npz   compare_test_cases.generate_test_data + evaluate_dataset (:12-247) with
                       seeded np.random, constant and varying theta: the test sets and the
                       per-sample bilinear / ML metrics of the reference's fp32 CPU model
  cascade20_fixture.npz  config #5 exactly (20 -> 640, five 2x applies) with bounded weights (the
                       fixture state, final.weight x 1e-3: the residual dominates, every level stays
                       in the physical range), strided 320^2 / 640^2 outputs and their metrics

Usage: ``make_golden.py [name ...]`` (default: the four fast fixtures; ``unet_b1024`` and
``cascade640`` take minutes and are generated on request).
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
sys.modules["seaborn"].kdeplot = lambda *a, **k: None     # plot-only (compare_test_cases.py:225-226)

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


B1024_SAMPLE_K = 256
B1024_CKPT = ["enc1", "enc2", "enc3", "bridge", "att3", "dec3", "att2", "dec2", "att1", "dec1"]


def _b1024_run(tag):
    """One reference train step at B=1024 in fp64 ("64") or fp32 ("32"); returns a dict of arrays."""
    import functools
    from torch.utils.checkpoint import checkpoint
    torch.set_num_threads(os.cpu_count())
    dt = torch.float64 if tag == "64" else torch.float32
    x, t = fixture_inputs(1024, seed=11)
    m = ref_model(dt).train()
    if tag == "64":
        for name in B1024_CKPT:
            mod = getattr(m, name)
            mod.forward = functools.partial(checkpoint, mod.forward, use_reentrant=False)
    xx = torch.from_numpy(x).to(dt)
    y = m(xx)
    loss = torch.nn.MSELoss()(y, torch.from_numpy(t).to(dt))
    out = {}
    # BN running stats after the forward, before a checkpoint recompute updates them again
    for k, v in m.state_dict().items():
        if k.endswith("running_mean") or k.endswith("running_var"):
            out[f"rs{tag}:{k}"] = v.double().numpy().copy()
    yf = y.detach().reshape(-1)
    idx = np.arange(0, yf.numel(), 97, dtype=np.int64)
    out["out_idx"] = idx
    out[f"out{tag}"] = yf[idx].double().numpy()
    out[f"out_sum{tag}"] = y.detach().double().sum(dim=(1, 2, 3)).numpy()
    out[f"out_sq{tag}"] = (y.detach().double() ** 2).sum(dim=(1, 2, 3)).numpy()
    out[f"loss{tag}"] = np.array(loss.item())
    loss.backward()
    names = trainable_names()
    params = dict(m.named_parameters())
    gn = []
    for i, n in enumerate(names):
        g = params[n].grad.detach().reshape(-1)
        gn.append(float(torch.linalg.vector_norm(g.double())))
        gi = sample_indices(g.numel(), 5000 + i, k=B1024_SAMPLE_K)
        out[f"gidx:{n}"] = gi
        out[f"gval{tag}:{n}"] = g[gi].double().numpy()
    out[f"gnorm{tag}"] = np.array(gn)
    # one clip + AdamW step exactly as train_enhanced.py:74-75, 308
    opt = torch.optim.AdamW(m.parameters(), lr=2e-4, weight_decay=1e-4)
    tot = torch.nn.utils.clip_grad_norm_(m.parameters(), 1.0)
    out[f"clip_total{tag}"] = np.array(float(tot))
    opt.step()
    for n in names:
        p = params[n].detach().reshape(-1)
        out[f"pval{tag}:{n}"] = p[out[f"gidx:{n}"]].double().numpy()
    return out


def unet_b1024_fixture():
    """Config #2 at full size (B=1024, train mode).  fp64 and fp32 run in separate child
    processes (each needs ~20 GB of host memory)."""
    import subprocess
    import tempfile
    merged = {"B": np.array(1024), "input_seed": np.array(11)}
    with tempfile.TemporaryDirectory() as td:
        for tag in ("64", "32"):
            dst = os.path.join(td, f"b{tag}.npz")
            subprocess.run([sys.executable, os.path.abspath(__file__), f"_b1024:{tag}:{dst}"], check=True)
            with np.load(dst) as z:
                merged.update({k: z[k] for k in z.files})
    np.savez_compressed(os.path.join(HERE, "unet_b1024_fixture.npz"), **merged)


def cascade640_fixture():
    """Config #5's cascade pinned to 640^2, with the paired interpolation baselines."""
    import resolution_comparison_enhanced as ref_rce
    torch.set_num_threads(os.cpu_count())
    np.random.seed(0)
    data = ref_rc.solve_multi_resolution(40, [80, 160, 320, 640])
    m = ref_model(torch.float32).eval()
    out = {"k1": np.array(data["k1"]), "k2": np.array(data["k2"]), "u40": data["u"][40]}
    sub = {80: (1, 1), 160: (1, 1), 320: (2, 3), 640: (3, 5)}   # stored grid strides (rows, cols)
    for r in (40, 80, 160, 320, 640):
        u = data["u"][r]
        out[f"u{r}_stats"] = np.array([u.mean(), u.std(), np.linalg.norm(u), u.min(), u.max()])
        out[f"u{r}_row"] = u[r // 3].copy()
    for tgt in (80, 160, 320, 640):
        ml = ref_rc.ml_multi_level_upscale(m, data, tgt, "cpu")
        out[f"ml{tgt}"] = ml.astype(np.float32) if tgt >= 320 else ml
        u40 = torch.from_numpy(data["u"][40]).float()[None, None]
        sols = {
            "blm": ref_rce.bilinear_multi_level_upscale(data, tgt),
            "cbm": ref_rce.cubic_multi_level_upscale(data, tgt),
            "bld": torch.nn.functional.interpolate(u40, size=(tgt, tgt), mode="bilinear",
                                                   align_corners=True).squeeze().numpy(),
            "cbd": torch.nn.functional.interpolate(u40, size=(tgt, tgt), mode="bicubic",
                                                   align_corners=True).squeeze().numpy(),
            "ml": ml,
        }
        sr, sc = sub[tgt]
        for k, v in sols.items():
            e = v - data["u"][tgt]
            out[f"{k}{tgt}_metrics"] = np.array([np.mean(np.abs(e)), np.sqrt(np.mean(e ** 2))])
            if k != "ml":
                out[f"{k}{tgt}"] = v[::sr, ::sc].copy()
    # config #5 starts at 20^2 (five 2x applies).  The reference hard-codes 40 as the start
    # (resolution_comparison.py:188), so its 20 -> 40 level is composed from its own
    # upscale_subdomain with the GT-statistics normalisation its level loop uses (:196-201), and
    # the loop then runs from that 40^2 prediction.  Same seed, so the same 640^2 (f, theta).
    np.random.seed(0)
    d20 = ref_rc.solve_multi_resolution(20, [40, 80, 160, 320, 640])
    gn = ref_rc.GlobalNormalization(d20["u"][40], d20["u"][20], d20["f"][40], d20["theta"][40])
    u40 = ref_rc.upscale_subdomain(m, d20["u"][20], d20["f"][40], d20["theta"][40], gn, "cpu")
    d20m = dict(d20)
    d20m["u"] = dict(d20["u"])
    d20m["u"][40] = u40
    ml = ref_rc.ml_multi_level_upscale(m, d20m, 640, "cpu")
    e = ml - d20["u"][640]
    out["ml640_from20"] = ml[::3, ::5].astype(np.float32)
    out["ml640_from20_metrics"] = np.array([np.mean(np.abs(e)), np.sqrt(np.mean(e ** 2))])
    out["u20"] = d20["u"][20]
    np.savez_compressed(os.path.join(HERE, "cascade640_fixture.npz"), **out)


def init_fixture():
    """M10: the reference's seeded initialisation (models.py:209-222 applied after seed 42)."""
    torch.manual_seed(42)
    m = ref_models.UNet()
    m.apply(ref_models.init_weights)
    out = {}
    for k, v in m.state_dict().items():
        f = v.detach().reshape(-1).double()
        if v.is_floating_point():
            out[f"norm:{k}"] = np.array(float(f.norm()))
            out[f"sum:{k}"] = np.array(float(f.sum()))
            out[f"sample:{k}"] = f[:: max(1, f.numel() // 64)][:64].numpy()
        else:
            out[f"int:{k}"] = v.numpy()
    np.savez_compressed(os.path.join(HERE, "init_fixture.npz"), **out)


def report_fixture():
    """compare_test_cases.py:12-247 on seeded draws (it writes data/*.npz and PNGs: run in a
    scratch directory)."""
    import tempfile
    from pathlib import Path
    import compare_test_cases as ref_ct
    m = ref_model(torch.float32).eval()
    out = {}
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as td:
        os.chdir(td)
        try:
            for tag, const in (("const", True), ("var", False)):
                np.random.seed(3)
                d = ref_ct.generate_test_data((1.0, 6.0), 6, f"t_{tag}", constant_theta=const)
                for key in ("k1", "k2", "u_fine", "u_coarse", "theta_fine", "theta_coarse", "f_fine"):
                    out[f"{tag}:{key}"] = np.asarray(d[key])
                metrics, avg = ref_ct.evaluate_dataset(d, m, "cpu", Path(td), f"t_{tag}")
                out[f"{tag}:metrics"] = np.array([[mm[k] for k in ("bilinear_mae", "bilinear_rmse", "ml_mae",
                                                                     "ml_rmse")] for mm in metrics])
                out[f"{tag}:avg"] = np.array([avg[k] for k in ("avg_bilinear_mae", "avg_bilinear_rmse",
                                                               "avg_ml_mae", "avg_ml_rmse")])
        finally:
            os.chdir(cwd)
    np.savez_compressed(os.path.join(HERE, "report_fixture.npz"), **out)


CASCADE20_FINAL_SCALE = 1e-3


def cascade20_fixture():
    """Config #5 at the physical bar: 20 -> 640 with the fixture weights, final.weight scaled by
    1e-3 so that the residual path dominates and the cascade stays physical at every level (with
    the raw random weights each level feeds an O(1) prediction back, resolution_comparison.py:191-226).
    The reference hard-codes 40 as the start (:188): its 20 -> 40 level is composed from its own
    upscale_subdomain with the level loop's GT normalisation (:196-201), as cascade640_fixture does."""
    torch.set_num_threads(os.cpu_count())
    m = ref_model(torch.float32).eval()
    with torch.no_grad():
        m.final.weight.mul_(CASCADE20_FINAL_SCALE)
    np.random.seed(0)
    d20 = ref_rc.solve_multi_resolution(20, [40, 80, 160, 320, 640])
    gn = ref_rc.GlobalNormalization(d20["u"][40], d20["u"][20], d20["f"][40], d20["theta"][40])
    u40 = ref_rc.upscale_subdomain(m, d20["u"][20], d20["f"][40], d20["theta"][40], gn, "cpu")
    out = {"u20": d20["u"][20], "ml40": u40, "final_scale": np.array(CASCADE20_FINAL_SCALE)}
    for tgt, (sr, sc) in ((80, (1, 1)), (160, (1, 1)), (320, (2, 3)), (640, (3, 5))):
        d = dict(d20)
        d["u"] = dict(d20["u"])
        d["u"][40] = u40
        ml = ref_rc.ml_multi_level_upscale(m, d, tgt, "cpu")
        e = ml - d20["u"][tgt]
        out[f"ml{tgt}"] = ml[::sr, ::sc].copy()
        out[f"ml{tgt}_metrics"] = np.array([np.mean(np.abs(e)), np.sqrt(np.mean(e ** 2))])
    np.savez_compressed(os.path.join(HERE, "cascade20_fixture.npz"), **out)


FIXTURES = {"init": init_fixture, "report": report_fixture, "cascade20": cascade20_fixture,
            "unet": unet_fixture, "poisson": poisson_fixture, "datagen": datagen_fixture,
            "cascade": cascade_fixture, "unet_b1024": unet_b1024_fixture, "cascade640": cascade640_fixture}

if __name__ == "__main__":
    args = sys.argv[1:]
    if args and args[0].startswith("_b1024:"):
        _, tag, dst = args[0].split(":", 2)
        np.savez(dst, **_b1024_run(tag))
        sys.exit(0)
    for name in args or ["unet", "poisson", "datagen", "cascade"]:
        FIXTURES[name]()
    for f in sorted(os.listdir(HERE)):
        print(f, os.path.getsize(os.path.join(HERE, f)))
