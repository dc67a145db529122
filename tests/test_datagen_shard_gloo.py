"""CPU, world_size 2 over gloo: sharded data generation (SURVEY 8(e) data-gen row).

Every rank draws the whole random sequence (k1, k2[, start_x, start_y] per sample, global
np.random) so the seeded dataset is unchanged, solves only its contiguous slice, and one
all-gather per field assembles the full set.  The HIP solver cannot run here, so the test swaps
the two device entry points (forcing, CG solve) for the oracle (scipy spsolve) -- the sharding,
draw order and gather are the code under test; the solver itself is pinned on the GPU
(tests/test_gpu_poisson.py).  Reference: data_generation.py:106-159,
enhanced_data_generation.py:98-191."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cpu_solver(monkey_target):
    from oracle import poisson_ref as R

    def forcing_batched(k12, n, device="cpu"):
        k = np.asarray(k12, dtype=np.float64).reshape(-1, 2)
        return torch.from_numpy(np.stack([R.forcing(a, b, n) for a, b in k])) if len(k) else \
            torch.empty(0, n, n, dtype=torch.float64)

    def solve_batched(f, theta, device="cpu", **kw):
        f = torch.as_tensor(f, dtype=torch.float64)
        theta = torch.as_tensor(theta, dtype=torch.float64).expand_as(f)
        return torch.from_numpy(np.stack([R.solve(a.numpy(), t.numpy()) for a, t in zip(f, theta)])) if len(f) else \
            torch.empty_like(f)

    monkey_target.forcing_batched = forcing_batched
    monkey_target.solve_batched = solve_batched


def _generate(shard, sizes=(5, 3)):
    from superresolution_for_pdes_amd import poisson as P
    from superresolution_for_pdes_amd.enhanced_data_generation import EnhancedPoissonSolver
    _cpu_solver(P)
    s = EnhancedPoissonSolver(20, 40, 80, device="cpu")
    np.random.seed(123)
    d1 = s.generate_dataset(n_samples=sizes[0], k_range=(0.5, 5.0), keep_on_device=True, shard=shard)
    d2 = s.generate_subdomain_dataset(n_samples=sizes[1], k_range=(0.5, 12.0), keep_on_device=True, shard=shard)
    after = np.random.uniform()           # the RNG stream must be where the single-process run leaves it
    return s.combine_datasets(d1, d2), after


def _worker(rank, world, port, q, sizes=(5, 3)):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        data, after = _generate(None, sizes)      # shard from the process group
        want, want_after = _generate((0, 1), sizes)
        same = set(data) == set(want) and all(
            np.array_equal(np.asarray(data[k]), np.asarray(want[k])) for k in want)
        q.put((rank, same, after == want_after, len(data["u_fine"])))
    finally:
        dist.destroy_process_group()


def test_sharded_datagen_equals_single_process_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(world)])
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, same, rng_ok, n in res:
        assert same, rank
        assert rng_ok, rank
        assert n == 8


def test_sharded_datagen_with_empty_shards_world3():
    """n_samples < world: some ranks solve an empty slice and still join the gathers."""
    world, sizes = 3, (2, 1)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q, sizes)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(world)])
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, same, rng_ok, n in res:
        assert same and rng_ok, rank
        assert n == 3


def test_shard_range_partitions():
    from superresolution_for_pdes_amd.data_generation import shard_range
    for n in (0, 1, 7, 1000, 1001):
        for world in (1, 2, 3, 8):
            parts = [shard_range(n, r, world) for r in range(world)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(parts, parts[1:]))
            assert max(h - l for l, h in parts) - min(h - l for l, h in parts) <= 1
