"""Config #4's data-parallel step with more than one rank, on the GPU.

Two fresh processes (torch.distributed.run) share the box's one GPU over gloo (RCCL refuses two
ranks on one device; the driver's 8-GPU run uses RCCL): the real U-Net DataParallel step at
per-rank batch 64 -- bucketed all-reduce overlapped with the backward, BN buffer broadcast,
FusedAdamW -- against each rank's single-process gradient (tests/ddp_step_worker.py).  The
reference loop this shards: src/train_enhanced.py:65-77."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _env():
    env = dict(os.environ)
    env["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    env.setdefault("OMP_NUM_THREADS", "4")
    return env


@pytest.mark.gpu
def test_data_parallel_unet_step_world2(tmp_path):
    out = tmp_path / "ddp.json"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(ROOT, "tests", "ddp_step_worker.py"), str(out), "64"]
    p = subprocess.run(cmd, env=_env(), capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    rec = json.loads(out.read_text())
    assert rec["world"] == 2 and rec["batch_per_rank"] == 64
    assert rec["ranks_differ"] > 1e-3                   # the two shards really give different gradients
    assert rec["grad_rel"] <= 1e-6, rec                 # all-reduced == mean of the single-process grads
    assert rec["grad_rel_max_tensor"] <= 1e-6, rec
    assert rec["n_buckets"] >= 4                        # bucketed (8 MB) while the backward ran
    assert rec["nbt_equal"] and rec["buffers_equal"], rec
    assert rec["params_equal"], rec                     # identical parameters after FusedAdamW


@pytest.mark.gpu
def test_bench_self_launches_ranks():
    """``bench.py --gpus 2`` without a launcher starts the two ranks itself and reports n_gpus 2
    (gloo here, see module docstring; SRPDE_BENCH_BACKEND selects it)."""
    env = _env()
    env["SRPDE_BENCH_BACKEND"] = "gloo"
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--batch", "64", "--no-cpu-baseline"]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["config"]["global_batch"] == 128
    assert rec["roofline"]["forward"]["train"]["ms"] > 0
