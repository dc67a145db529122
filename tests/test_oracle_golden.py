"""CPU: the oracle restatement is pinned against the golden vectors of the REAL reference
(tests/golden/make_golden.py ran reference src/ in the build container)."""
import numpy as np
import torch

from state import fixture_state_torch


def test_unet_oracle_matches_reference_forward(golden):
    from oracle import unet_ref as U
    z = golden["unet"]
    x = torch.from_numpy(z["x"])
    for tag, dt in (("32", torch.float32), ("64", torch.float64)):
        with torch.no_grad():
            out = U.unet_forward(U.clone_state(fixture_state_torch(dt)), x.to(dt), False)
        assert np.array_equal(out.numpy(), z[f"out_eval{tag}"]) or \
            np.max(np.abs(out.numpy() - z[f"out_eval{tag}"])) < 1e-12


def test_unet_oracle_matches_reference_train_step(golden):
    from oracle import unet_ref as U
    z = golden["unet"]
    x, t = torch.from_numpy(z["x"]), torch.from_numpy(z["t"])
    out, loss, grads, st = U.forward_with_grads(fixture_state_torch(torch.float64), x.double(), t.double())
    assert np.max(np.abs(out.numpy() - z["out_train64"])) < 1e-12
    assert abs(float(loss) - float(z["loss64"])) < 1e-12
    for k in z.files:
        if k.startswith("rs64:"):
            assert np.max(np.abs(st[k[5:]].numpy() - z[k])) < 1e-12
    for i, (n, g) in enumerate(grads.items()):
        idx = z[f"gidx:{n}"]
        assert np.max(np.abs(g.reshape(-1)[idx].numpy() - z[f"gval64:{n}"])) <= 1e-10 * max(1.0, z["gnorm64"][i])


def test_unet_oracle_adamw_step_matches_reference(golden):
    from oracle import unet_ref as U
    z = golden["unet"]
    x, t = torch.from_numpy(z["x"]), torch.from_numpy(z["t"])
    loss, new, grads, _, total = U.train_step(fixture_state_torch(torch.float32), x, t)
    assert abs(float(total) - float(z["clip_total32"])) < 1e-4 * float(z["clip_total32"])
    for n in grads:
        idx = z[f"gidx:{n}"]
        assert np.max(np.abs(new[n].reshape(-1)[idx].numpy() - z[f"pval32:{n}"])) < 1e-6, n


def test_poisson_oracle_matches_spsolve_fixtures(golden):
    from oracle import poisson_ref as R
    z = golden["poisson"]
    for n in (20, 40, 80):
        f = z[f"f{n}"]
        k1, k2 = z[f"k{n}"]
        assert np.max(np.abs(R.forcing(k1, k2, n) - f)) < 1e-15
        assert np.max(np.abs(R.solve(f, np.ones((n, n))) - z[f"u1_{n}"])) < 1e-15
        assert np.max(np.abs(R.solve(f, z[f"thv{n}"]) - z[f"uv_{n}"])) < 1e-15
        u, it = R.cg(f, z[f"thv{n}"])
        assert np.linalg.norm(u - z[f"uv_{n}"]) / np.linalg.norm(z[f"uv_{n}"]) < 1e-10
        assert it < 10 * n


def test_datagen_oracle_matches_reference(golden):
    from oracle import poisson_ref as R
    z = golden["datagen"]
    np.random.seed(123)
    d1 = R.generate_dataset(3, (0.5, 5.0))
    np.random.seed(7)
    d2 = R.generate_subdomain(3, (0.5, 12.0))
    for k, v in d1.items():
        assert np.allclose(v, z[f"std:{k}"], rtol=0, atol=1e-14), k
    for k, v in d2.items():
        assert np.allclose(v, z[f"sub:{k}"], rtol=0, atol=1e-14), k
    comb = R.combine(dict(d1), d2)
    for k, v in comb.items():
        assert np.allclose(v, z[f"comb:{k}"], rtol=0, atol=1e-14), k


def test_cascade_fixture_self_consistent(golden):
    """The cascade fixture's inputs follow solve_multi_resolution's seeded draw order."""
    from oracle import poisson_ref as R
    z = golden["cascade"]
    np.random.seed(0)
    d = R.solve_multi_resolution(40, (80, 160))
    assert d["k1"] == float(z["k1"]) and d["k2"] == float(z["k2"])
    for r in (40, 80, 160):
        assert np.array_equal(d["theta"][r], z[f"theta{r}"])
        assert np.max(np.abs(d["u"][r] - z[f"u{r}"])) < 1e-15


def test_interpolation_fixture_is_torch_interpolate(golden):
    """The cascade640 fixture's bilinear / bicubic baselines are aten's F.interpolate
    (align_corners=True) of the fp32 40^2 ground truth -- the semantics the HIP resize kernels
    restate (resolution_comparison_enhanced.py:19-65)."""
    import torch.nn.functional as F
    z = golden["cascade640"]
    u = torch.from_numpy(z["u40"]).float()[None, None]
    for mode, k in (("bilinear", "bld"), ("bicubic", "cbd")):
        for tgt, (sr, sc) in ((80, (1, 1)), (160, (1, 1)), (640, (3, 5))):
            v = F.interpolate(u, size=(tgt, tgt), mode=mode, align_corners=True)[0, 0].numpy()
            assert np.array_equal(v[::sr, ::sc], z[f"{k}{tgt}"])
