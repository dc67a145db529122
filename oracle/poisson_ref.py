"""numpy/scipy restatement of the reference Poisson data generation and cascade.

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).

Reference anchors:
* ``laplacian``              data_generation.py:35-58   DIA 5-point operator over all n^2
                                                         nodes, row-wrap links removed, /h^2
* ``solve``                  data_generation.py:79-104  spsolve(diag(theta) @ L, f)
* ``forcing``                data_generation.py:60-77   sin(2 pi k1 X) sin(2 pi k2 Y)
* ``generate_dataset``       data_generation.py:106-159
* ``generate_subdomain``     enhanced_data_generation.py:98-165 (+ extract/downsample :70-96)
* ``combine``                enhanced_data_generation.py:167-191
* ``solve_multi_resolution`` resolution_comparison.py:13-78
* ``split/stitch``           resolution_comparison.py:123-158
* ``global_stats``           resolution_comparison.py:160-181
* ``cascade``                resolution_comparison.py:80-121, 183-229
* ``cg``                     the matrix-free CG that the HIP kernel implements, on the
                             SPD form  (-L) u = -f / theta  (same solution as spsolve).
"""
from __future__ import annotations

import numpy as np
from scipy.sparse import diags
from scipy.sparse.linalg import spsolve


def laplacian(n: int):
    h = 1.0 / (n - 1)
    n2 = n * n
    main = -4.0 * np.ones(n2)
    off = np.ones(n2 - 1)
    off[np.arange(n - 1, n2 - 1, n)] = 0.0
    far = np.ones(n * (n - 1))
    return diags([main, off, off, far, far], [0, 1, -1, n, -n], shape=(n2, n2)) / (h * h)


def solve(f: np.ndarray, theta: np.ndarray) -> np.ndarray:
    n = f.shape[0]
    a = diags(theta.reshape(-1)) @ laplacian(n)
    return spsolve(a, f.reshape(-1)).reshape(n, n)


def apply_operator(u: np.ndarray, theta: np.ndarray) -> np.ndarray:
    """theta * (5-point Laplacian of u with a zero ghost ring) -- the matrix-free form."""
    n = u.shape[-1]
    h2 = (1.0 / (n - 1)) ** 2
    p = np.pad(u, [(0, 0)] * (u.ndim - 2) + [(1, 1), (1, 1)])
    lap = (p[..., :-2, 1:-1] + p[..., 2:, 1:-1] + p[..., 1:-1, :-2] + p[..., 1:-1, 2:] - 4.0 * u) / h2
    return theta * lap


def cg(f: np.ndarray, theta: np.ndarray, rtol: float = 1e-12, maxit: int = 100000):
    """Matrix-free CG on (-L) u = -f/theta; returns (u, iterations)."""
    b = -f / theta
    ones = np.ones_like(theta)
    x = np.zeros_like(b)
    r = b.copy()
    p = r.copy()
    rr = float(np.sum(r * r))
    stop = rtol * rtol * float(np.sum(b * b))
    it = 0
    while rr > stop and it < maxit:
        q = -apply_operator(p, ones)
        alpha = rr / float(np.sum(p * q))
        x += alpha * p
        r -= alpha * q
        rr_new = float(np.sum(r * r))
        p = r + (rr_new / rr) * p
        rr = rr_new
        it += 1
    return x, it


def grid(n: int):
    x = np.linspace(0, 1, n)
    return np.meshgrid(x, x)


def forcing(k1: float, k2: float, n: int) -> np.ndarray:
    X, Y = grid(n)
    return np.sin(2 * np.pi * k1 * X) * np.sin(2 * np.pi * k2 * Y)


def generate_dataset(n_samples, k_range=(1, 5), n_coarse=20, n_fine=40):
    ds = {k: [] for k in ("u_coarse", "u_fine", "f_coarse", "f_fine", "theta_coarse", "theta_fine", "k1", "k2")}
    for _ in range(n_samples):
        k1 = np.random.uniform(*k_range)
        k2 = np.random.uniform(*k_range)
        tf = np.ones((n_fine, n_fine))
        tc = np.ones((n_coarse, n_coarse))
        ff = forcing(k1, k2, n_fine)
        fc = forcing(k1, k2, n_coarse)
        ds["u_fine"].append(solve(ff, tf))
        ds["u_coarse"].append(solve(fc, tc))
        ds["f_coarse"].append(fc)
        ds["f_fine"].append(ff)
        ds["theta_coarse"].append(tc)
        ds["theta_fine"].append(tf)
        ds["k1"].append(k1)
        ds["k2"].append(k2)
    return {k: np.array(v) for k, v in ds.items()}


def generate_subdomain(n_samples, k_range=(0.5, 12.0), n_fine=40, n_superfine=80):
    ds = {k: [] for k in ("u_coarse", "u_fine", "f_coarse", "f_fine", "theta_coarse", "theta_fine",
                          "k1", "k2", "is_subdomain")}
    for _ in range(n_samples):
        k1 = np.random.uniform(*k_range)
        k2 = np.random.uniform(*k_range)
        ts = np.ones((n_superfine, n_superfine))
        fs = forcing(k1, k2, n_superfine)
        us = solve(fs, ts)
        sx = np.random.randint(0, n_superfine - n_fine)
        sy = np.random.randint(0, n_superfine - n_fine)
        cut = lambda a: a[sy:sy + n_fine, sx:sx + n_fine]
        tf, ff, uf = cut(ts), cut(fs), cut(us)
        ds["u_coarse"].append(uf[::2, ::2])
        ds["u_fine"].append(uf)
        ds["f_coarse"].append(ff[::2, ::2])
        ds["f_fine"].append(ff)
        ds["theta_coarse"].append(tf[::2, ::2])
        ds["theta_fine"].append(tf)
        ds["k1"].append(k1)
        ds["k2"].append(k2)
        ds["is_subdomain"].append(True)
    return {k: np.array(v) for k, v in ds.items()}


def combine(d1, d2):
    if "is_subdomain" not in d1:
        d1["is_subdomain"] = np.zeros(len(d1["u_fine"]), dtype=bool)
    return {k: (np.concatenate([d1[k], d2[k]]) if k in d2 else d1[k]) for k in d1}


def solve_multi_resolution(n_coarse=40, resolutions=(80, 160, 320, 640)):
    k1 = np.random.uniform(10.0, 11.0)
    k2 = np.random.uniform(10.0, 11.0)
    nf = max(resolutions)
    X, Y = grid(nf)
    f_fin = np.sin(k1 * 2 * np.pi * X) * np.sin(k2 * 2 * np.pi * Y)
    th_fin = np.random.uniform(0.5, 2.0, size=(nf, nf))
    data = {"k1": k1, "k2": k2, "f": {}, "theta": {}, "u": {}}
    for res in [n_coarse] + list(resolutions):
        step = nf // res
        data["f"][res] = f_fin if res == nf else f_fin[::step, ::step]
        data["theta"][res] = th_fin if res == nf else th_fin[::step, ::step]
        data["u"][res] = solve(data["f"][res], data["theta"][res])
    return data


def split(a, s):
    m = a.shape[0] // s
    return [[a[i * s:(i + 1) * s, j * s:(j + 1) * s] for j in range(m)] for i in range(m)]


def stitch(tiles):
    s = tiles[0][0].shape[0]
    out = np.zeros((len(tiles) * s, len(tiles[0]) * s))
    for i, row in enumerate(tiles):
        for j, t in enumerate(row):
            out[i * s:(i + 1) * s, j * s:(j + 1) * s] = t
    return out
