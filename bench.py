#!/usr/bin/env python3
"""Headline benchmark: 20->40 SR training samples/s at batch 1024 per GPU (BASELINE.json).

One "step" = the reference's inner training step (src/train_enhanced.py:68-75) on one
batch of 1024 synthetic 40x40 fields resident in HBM: HIP U-Net forward (train-mode BN),
HIP MSE, HIP backward, RCCL gradient all-reduce (N>1, overlapped with backward), fused
clip_grad_norm_(1.0) + AdamW(lr 2e-4, wd 1e-4).  Nothing is skipped in the timed region.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...      (one process per GPU, RCCL)

Rank 0 prints ONE JSON line.  ``roofline`` prices the dominant kernel (the implicit-GEMM
conv forward of the layer named by --roofline-layer) from HIP events recorded around its
launch on the compute stream; ``cpu_baseline`` times the oracle (torch-CPU restatement of
the same step) on the host cores for a bounded sample.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FWD_GFLOP_PER_SAMPLE = None  # computed from the architecture table below

# dense 3x3 conv layers of the U-Net: (name, cin, cout, hw)  -- models.py:36-60
CONV3 = [("enc1.conv1", 3, 64, 40), ("enc1.conv2", 64, 64, 40), ("enc2.conv1", 64, 128, 20),
         ("enc2.conv2", 128, 128, 20), ("enc3.conv1", 128, 256, 10), ("enc3.conv2", 256, 256, 10),
         ("bridge.0", 256, 512, 10), ("bridge.3", 512, 512, 10), ("dec3.conv1", 768, 256, 10),
         ("dec3.conv2", 256, 256, 10), ("dec2.conv1", 384, 128, 20), ("dec2.conv2", 128, 128, 20),
         ("dec1.conv1", 192, 64, 40), ("dec1.conv2", 64, 64, 40), ("out_conv1", 64, 32, 40),
         ("out_conv2", 32, 16, 40)]


_JSON_OUT = None


def emit(rec):
    """The one JSON line, on the process's original stdout (see main: library banners such as
    RCCL's version block are moved to stderr so stdout carries only this line)."""
    out = _JSON_OUT or sys.stdout
    out.write(json.dumps(rec) + "\n")
    out.flush()


def conv_flops(cin, cout, hw):
    return 2.0 * cout * cin * 9 * hw * hw


# whole-forward algorithmic cost per sample, SURVEY 3.4 / 8(d) [measured on the reference]:
# 26 conv calls = 2.6753 GFLOP; unfused fp32 activation traffic (every op's inputs + outputs,
# weights excluded) = 36.31 MB.  north_star's target: >= 60 % of the HBM roofline on this forward
FWD_FLOP_PER_SAMPLE = 2.6753e9
FWD_BYTES_PER_SAMPLE = 36.31e6
HBM_PEAK = 8.0e12


def default_traffic_json():
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "traffic_r*.json")))
    return files[-1] if files else None


def time_forward(model, x, training, reps=10, warm=3):
    """Average ms of one B-sample U-Net forward (no autograd), HIP events on the stream it runs on.
    Train mode is the step's forward (batch statistics, running-stat update, the stored operand
    splits the weight gradient reads); eval mode is inference (running statistics, cached weight
    split)."""
    was = model.training
    model.train(training)
    st = torch.cuda.current_stream(x.device)
    with torch.no_grad():
        for _ in range(warm):
            model(x)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        for _ in range(reps):
            model(x)
        b.record(st)
        b.synchronize()
    model.train(was)
    return a.elapsed_time(b) / reps


def forward_roofline(model, x, peak_tf):
    """roofline.forward: the north-star figure (>= 60 % of HBM roofline on the B=1024 40x40 forward,
    i.e. forward <= 7.75 ms), with the MFMA fraction beside it."""
    B = x.shape[0]
    out = {"batch": B, "algorithmic_bytes": FWD_BYTES_PER_SAMPLE * B, "algorithmic_flop": FWD_FLOP_PER_SAMPLE * B,
           "hbm_peak_gbs": HBM_PEAK / 1e9, "mfma_peak_tflops": peak_tf,
           "target": "hbm_frac >= 0.60 (forward <= %.2f ms)" % (FWD_BYTES_PER_SAMPLE * B / (0.6 * HBM_PEAK) * 1e3)}
    for mode, training in (("train", True), ("eval", False)):
        ms = time_forward(model, x, training)
        t = ms * 1e-3
        out[mode] = {"ms": round(ms, 4), "samples_per_s": round(B / t, 1),
                     "hbm_gbs": round(FWD_BYTES_PER_SAMPLE * B / t / 1e9, 1),
                     "hbm_frac": round(FWD_BYTES_PER_SAMPLE * B / t / HBM_PEAK, 4),
                     "tflops": round(FWD_FLOP_PER_SAMPLE * B / t / 1e12, 2),
                     "mfma_frac": round(FWD_FLOP_PER_SAMPLE * B / t / 1e12 / peak_tf, 4)}
    return out


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=1024, help="per-GPU batch (BASELINE config: 1024)")
    ap.add_argument("--roofline-layer", default="bridge.3")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-live-traffic", action="store_true",
                    help="skip the two rocprofv3 PMC passes that measure the roofline kernel's HBM bytes for this "
                         "line (N=1 train only) and take them from --traffic-json / the newest profiles file")
    ap.add_argument("--traffic-json", default=None,
                    help="PMC traffic of the roofline kernel (tools/traffic_json.py output); default: the newest "
                         "profiles/traffic_r*.json, which round_evidence.sh measures on the tree it commits with")
    ap.add_argument("--workload", choices=("train", "poisson", "cascade"), default="train",
                    help="train = the BASELINE metric (default); poisson = config #3 CG data-gen solve; "
                         "cascade = config #5 20->640 multi-level inference")
    ap.add_argument("--poisson-sizes", default="40:1024,80:1024,160:64,320:16,640:4",
                    help="n:B pairs for --workload poisson")
    ap.add_argument("--checkpoint", default=None, help="--workload cascade: model_state_dict checkpoint")
    ap.add_argument("--cascade-fixture", default=None,
                    help="--workload cascade: the reference's 20->640 output for these weights (npz key ml640_from20, "
                         "every 3rd row / 5th column; tests/golden/cascade640_fixture.npz with the cascade20 state)")
    ap.add_argument("--ddp", action="store_true",
                    help="use the process group + DataParallel path even at world size 1 (RCCL smoke check)")
    ap.add_argument("--ddp-rccl", action="store_true",
                    help="with --ddp at world size 1: keep the buckets' one-rank RCCL all-reduce (by default a "
                         "one-rank group skips it), so the step carries RCCL's kernels and stream")
    return ap.parse_args()


def host_threads():
    """All host cores this process may use: the box's CPU share (OMP_NUM_THREADS, 16 per GPU on the
    pool) -- os.cpu_count() there reports the whole machine."""
    env = os.environ.get("OMP_NUM_THREADS")
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    return max(1, min(n, int(env))) if env and env.isdigit() else n


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(seconds):
    """Oracle (torch-CPU restatement of UNet + MSE + backward + clip + AdamW) on the host cores,
    as BASELINE.md section 3 / SURVEY 8(d) prescribe: all cores, 2 warm-ups, then the median of
    >= 5 timed steps (time.perf_counter) at the reference's batch 32.  Also config #1 as the
    reference runs it: train_model for one epoch on 64 samples (80/20 split, batch 32: two train
    steps on 51 samples, one eval batch of 13), median of 3 epochs."""
    import statistics
    from oracle import unet_ref as U
    threads = host_threads()
    torch.set_num_threads(threads)
    st = U.kaiming_init_state(0)
    b = 32
    g = torch.Generator().manual_seed(1)
    x = torch.randn(64, 3, 40, 40, generator=g)
    x[:, 1] = 1.0
    t = torch.randn(64, 1, 40, 40, generator=g)
    opt, step = None, 0
    for _ in range(2):   # warm-ups
        step += 1
        _, st, _, opt, _ = U.train_step(st, x[:b], t[:b], opt_state=opt, step=step)
    times, t_all = [], time.perf_counter()
    while len(times) < 5 or (time.perf_counter() - t_all < 0.6 * seconds and len(times) < 200):
        step += 1
        t0 = time.perf_counter()
        _, st, _, opt, _ = U.train_step(st, x[:b], t[:b], opt_state=opt, step=step)
        times.append(time.perf_counter() - t0)
    med = statistics.median(times)
    # config #1: one train_model epoch on 64 samples (train_enhanced.py:60-92 with the oracle step)
    tr, va = slice(0, 51), slice(51, 64)
    epochs = []
    for _ in range(4):
        t0 = time.perf_counter()
        for lo in range(0, 51, b):
            step += 1
            sl = slice(lo, min(lo + b, 51))
            _, st, _, opt, _ = U.train_step(st, x[tr][sl], t[tr][sl], opt_state=opt, step=step)
        with torch.no_grad():
            torch.nn.functional.mse_loss(U.unet_forward(st, x[va], False), t[va])
        epochs.append(time.perf_counter() - t0)
    ep = statistics.median(epochs[1:])
    return {"value": round(b / med, 2), "unit": "samples/s", "cores": threads, "kind": "port",
            "cpu": cpu_model(),
            "sample": f"median of {len(times)} oracle train steps (fwd+MSE+bwd+clip+AdamW) at batch {b} after 2 "
                      f"warm-ups: {1e3 * med:.1f} ms/step; config #1 (train_model epoch, 64 samples, batch 32, "
                      f"+ val): {ep:.3f} s/epoch = {51 / ep:.1f} train samples/s (median of 3 after 1 warm-up); "
                      f"torch {torch.__version__}, {threads} threads",
            "config1_epoch_s": round(ep, 4)}


def cpu_baseline_poisson(seconds, sizes=(40, 80)):
    """Oracle spsolve (the reference's SciPy SuperLU call) per problem on the host."""
    import numpy as np
    from oracle import poisson_ref as R
    out, rng = {}, np.random.default_rng(7)
    per = seconds / len(sizes)
    for n in sizes:
        k = rng.uniform(0.5, 12.0, 2)
        f = R.forcing(k[0], k[1], n)
        th = rng.uniform(0.5, 2.0, (n, n))
        R.solve(f, th)
        cnt, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < per or cnt < 2:
            R.solve(f, th)
            cnt += 1
        out[n] = cnt / (time.perf_counter() - t0)
    return out


def measure_traffic_poisson(sizes):
    """HBM bytes per launch of the Poisson kernels (cg_lds_kernel, gcg_coop_kernel), measured now:
    two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; --kernel-trace only) over this script solving
    `sizes` once, FETCH_SIZE doubled (MI355X_MICROARCH.md's gfx950 correction).  Child processes under
    a hard time limit, started before this process touches the GPU.  -> dict or None."""
    import csv
    import glob
    import shutil
    import subprocess
    import tempfile
    prof = shutil.which("rocprofv3")
    if prof is None:
        return {"error": "rocprofv3 not found"}
    d = tempfile.mkdtemp(prefix="srpde_pmc_", dir="/tmp")
    env = dict(os.environ, TMPDIR="/tmp")
    exit_fault = None
    try:
        for i, c in enumerate(("FETCH_SIZE", "WRITE_SIZE")):
            cmd = ["timeout", "-s", "KILL", "120", prof, "--pmc", c, "--kernel-trace", "--output-format", "csv",
                   "-d", d, "-o", f"p{i}", "--", sys.executable, os.path.abspath(__file__), "--workload", "poisson",
                   "--poisson-sizes", sizes, "--steps", "1", "--no-cpu-baseline", "--no-live-traffic"]
            r = subprocess.run(cmd, cwd="/tmp", env=env, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)
            wrote = bool(glob.glob(f"{d}/**/p{i}_counter_collection.csv", recursive=True))
            if r.returncode != 0 and not (wrote and "tool finalization" in r.stderr):
                return {"error": f"PMC pass {c} rc {r.returncode}: {r.stderr[-300:]}"}
            if r.returncode != 0:   # the exit-time fault after the counters were written (see the caller)
                exit_fault = f"pass {c}: rc {r.returncode} after rocprofv3 wrote its counters"
        vals = {}
        for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                for k in ("cg_lds", "gcg_coop_kernel"):   # cg_lds_kernel<NPT> / cg_lds_n_kernel<N, T>
                    if k in r["Kernel_Name"]:
                        vals.setdefault((k, r["Counter_Name"]), []).append(float(r["Counter_Value"]))
        out = {"sizes": sizes}
        for k in ("cg_lds", "gcg_coop_kernel"):
            fe, wr = vals.get((k, "FETCH_SIZE")), vals.get((k, "WRITE_SIZE"))
            if fe and wr:
                out[k] = round(1024 * (2 * sum(fe) / len(fe) + sum(wr) / len(wr)))
        if len(out) == 1:
            out["error"] = f"no counter rows for the CG kernels ({len(vals)} series)"
        if exit_fault:
            out["exit_fault"] = exit_fault
        return out
    except Exception as e:   # noqa: BLE001 -- the bench line must not depend on the profiler
        return {"error": f"PMC measurement failed: {e}"}
    finally:
        shutil.rmtree(d, ignore_errors=True)


def run_poisson(args, world, rank, dev, pmc=None):
    """Config #3: batched on-device CG (HIP) solves/s.  Each rank solves its own B problems
    per size (independent units, weak scaling, no collective)."""
    import numpy as np
    from superresolution_for_pdes_amd import poisson as P
    sizes = [tuple(int(v) for v in s.split(":")) for s in args.poisson_sizes.split(",")]
    rng = np.random.default_rng(100 + rank)
    levels = {}
    for n, B in sizes:
        k = rng.uniform(0.5, 12.0, (B, 2))
        f = P.forcing_batched(k, n, device=dev)
        th = torch.from_numpy(rng.uniform(0.5, 2.0, (B, n, n))).to(dev)
        u, it = P.solve_batched(f, th, device=dev, return_iters=True)   # warm-up (+ iteration counts)
        reps = max(1, min(args.steps, 5 if n >= 320 else args.steps))
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            u, it = P.solve_batched(f, th, device=dev, return_iters=True)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        if world > 1:
            tt = torch.tensor([el], device=dev, dtype=torch.float64)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            el = float(tt)
        iters = float(it.double().mean())
        t = el / reps
        pts_it = B * n * n * iters
        lv = {"B": B, "solves_per_s": round(world * B / t, 2), "ms_per_batch": round(1e3 * t, 3),
              "mean_iters": round(iters, 1)}
        if n <= 128:   # LDS-resident: fp64 VALU bound, 19 flop / point / iteration
            lv["fp64_tflops"] = round(19 * pts_it / t / 1e12, 3)
            lv["fp64_frac"] = round(19 * pts_it / t / 78.6e12, 4)
        else:
            # grid CG: every point's state stays on chip for the whole solve (registers + LDS, DESIGN
            # 3.6), so HBM moves only f, theta, u (24 B / point / solve) and the edge rows exchanged per
            # iteration; the bound is the iteration's latency chain (one grid barrier + two round
            # trips), reported per iteration of the slowest problem in the batch
            lv["max_iters"] = int(it.max())
            lv["us_per_iter"] = round(1e6 * t / max(1, int(it.max())), 2)
            # SURVEY 8(d)'s convention for a streamed CG (88 B / point / iteration: SpMV, updates and
            # direction through HBM): the rate this solve equals under it (above 1 of the HBM peak because
            # the state never leaves the chip)
            lv["hbm_equiv_gbs_88B"] = round(88 * pts_it / t / 1e9, 1)
            lv["hbm_equiv_frac_88B"] = round(88 * pts_it / t / 8.0e12, 4)
        levels[n] = lv
    if rank != 0:
        return
    hn = 80 if 80 in levels else min(levels)
    head = levels[hn]
    rec = {"metric": "Poisson CG solves/s (batched fp64 5-point, rtol 1e-12)",
           "value": head["solves_per_s"], "unit": "solves/s", "n_gpus": world, "steps": args.steps,
           "warmup": 1, "ms_per_step": head["ms_per_batch"], "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": "f64",
           "data": "synthetic: f = sin(2 pi k1 x) sin(2 pi k2 y), k ~ U(0.5,12), theta ~ U(0.5,2), in HBM",
           "config": {"workload": f"config #3 on-device data-gen solve, headline n={hn} B={head['B']}/GPU",
                      "levels": {str(k): v for k, v in levels.items()}}}
    if hn <= 128:   # the headline kernel: the LDS-resident CG, fp64 VALU bound (dense fp64 vector peak)
        rec["roofline"] = {"bound": "fp64-valu",
                           "kernel": "cg_lds_n_kernel<80, 960>" if hn == 80 else f"cg_lds_kernel[n={hn}]",
                           "achieved": head["fp64_tflops"],
                           "peak": 78.6, "unit": "TFLOP/s", "frac": head["fp64_frac"],
                           "traffic": (pmc or {}).get("cg_lds"),
                           "traffic_note": "HBM bytes per launch (one batch), rocprofv3 FETCH_SIZE x2 + WRITE_SIZE "
                                           "measured by this run; algorithmic 24 B per point (f, theta in, u out) = "
                                           f"{24 * head['B'] * hn * hn} B"}
        if pmc and pmc.get("error"):
            rec["roofline"]["traffic_note"] += f"; live measurement unavailable: {pmc['error']}"
        if pmc and pmc.get("gcg_coop_kernel"):
            rec["grid_cg_traffic"] = {"kernel": "gcg_coop_kernel", "bytes_per_launch": pmc["gcg_coop_kernel"],
                                      "sizes": pmc.get("sizes"),
                                      "note": "rocprofv3 FETCH_SIZE x2 + WRITE_SIZE (L2 <-> fabric requests): the "
                                              "grid barrier's polls and arrivals (device-scope atomics) dominate; "
                                              "the solve's own HBM data is f, theta, u and the edge rows",
                                      "exit_fault": pmc.get("exit_fault")}
    if not args.no_cpu_baseline and world == 1:
        cb = cpu_baseline_poisson(min(args.cpu_seconds, 10.0))
        rec["cpu_baseline"] = {"value": round(cb[80], 2), "unit": "solves/s", "cores": 1, "kind": "port",
                               "sample": "scipy spsolve(diag(theta) L, f) per problem (the reference's call), "
                                         + ", ".join(f"n={n}: {v:.1f}/s" for n, v in cb.items())}
    emit(rec)


def cpu_baseline_cascade(st, data, seconds):
    """The reference's cascade loop (batch-1 forwards, resolution_comparison.py:203-223) on
    the oracle U-Net, host cores; one full 20->640 pass (bounded by its own length)."""
    import numpy as np
    from oracle import unet_ref as U, poisson_ref as R
    import torch.nn.functional as F
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    t0 = time.perf_counter()
    cur, res, nf = np.asarray(data["u"][20]), 20, 0
    with torch.no_grad():
        while res < 640:
            nxt = 2 * res
            u32 = torch.tensor(np.asarray(data["u"][nxt]), dtype=torch.float32)
            f32 = torch.tensor(np.asarray(data["f"][nxt]), dtype=torch.float32)
            t32 = torch.tensor(np.asarray(data["theta"][nxt]), dtype=torch.float32)
            um, us, fm, fs, tm, ts = u32.mean(), u32.std(), f32.mean(), f32.std(), t32.mean(), t32.std()
            uc, ft, tt = R.split(cur, 20), R.split(np.asarray(data["f"][nxt]), 40), R.split(
                np.asarray(data["theta"][nxt]), 40)
            rows = []
            for ra, rb, rc in zip(uc, ft, tt):
                row = []
                for a, b, c in zip(ra, rb, rc):
                    x0 = F.interpolate(((torch.tensor(a, dtype=torch.float32) - um) / us)[None, None],
                                       size=(40, 40), mode="bilinear", align_corners=True)
                    x = torch.cat([x0, ((torch.tensor(c, dtype=torch.float32) - tm) / ts)[None, None],
                                   ((torch.tensor(b, dtype=torch.float32) - fm) / fs)[None, None]], 1)
                    row.append((U.unet_forward(st, x, training=False) * us + um)[0, 0].double().numpy())
                    nf += 1
                rows.append(row)
            cur, res = R.stitch(rows), nxt
            if time.perf_counter() - t0 > 4 * seconds:
                break
    dt = time.perf_counter() - t0
    return {"value": round(dt * 1e3, 1), "unit": "ms per 20->640 cascade", "cores": threads, "kind": "port",
            "sample": f"{nf} batch-1 oracle U-Net forwards (the reference's loop) in {dt:.2f}s, "
                      f"torch {torch.__version__} threads={threads}"}


def run_cascade(args, world, rank, dev):
    """Config #5: 20->640 multi-level cascade (5 levels; 256 tiles at the last), ground truth by
    the HIP CG at every resolution; subtrees sharded over ranks for N>1."""
    import numpy as np
    from superresolution_for_pdes_amd.models import UNet, init_weights
    from superresolution_for_pdes_amd import resolution_comparison as RC
    torch.manual_seed(42)
    model = UNet()
    model.apply(init_weights)
    if args.checkpoint:
        ck = torch.load(args.checkpoint, map_location="cpu", weights_only=True)
        model.load_state_dict(ck.get("model_state_dict", ck))
    model = model.to(dev).eval()
    np.random.seed(0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    data = RC.solve_multi_resolution(n_coarse=20, resolutions=(40, 80, 160, 320, 640), device=dev)
    torch.cuda.synchronize()
    gt_s = time.perf_counter() - t0
    dd = {k: {r: torch.as_tensor(v).to(dev) for r, v in data[k].items()} for k in ("u", "f", "theta")}
    for _ in range(max(1, args.warmup)):
        pred = RC.ml_multi_level_upscale(model, dd, 640, device=dev, start_resolution=20, return_tensor=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        pred = RC.ml_multi_level_upscale(model, dd, 640, device=dev, start_resolution=20, return_tensor=True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt)
    if rank != 0:
        return
    m = RC.cascade_metrics(pred.cpu().numpy(), data["u"][640])
    ref_err = None
    if args.cascade_fixture:
        ref = np.load(args.cascade_fixture)["ml640_from20"].astype(np.float64)
        pn = np.asarray(pred.cpu().numpy(), dtype=np.float64).reshape(640, 640)[::3, ::5]
        ref_err = float(np.sqrt(np.mean((pn - ref) ** 2)) / np.sqrt(np.mean(ref ** 2)))
    ms = 1e3 * el / args.steps
    tiles = 1 + 4 + 16 + 64 + 256
    rec = {"metric": "20->640 cascade latency (5 levels, 256 tiles at the last)", "value": round(ms, 3),
           "unit": "ms", "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 3),
           "higher_is_better": False, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
           "data": "synthetic: solve_multi_resolution seed 0 (k ~ U(10,11), theta ~ U(0.5,2)); "
                   + ("checkpoint " + os.path.basename(args.checkpoint) if args.checkpoint else "random-init U-Net"),
           "config": {"workload": "config #5 cascade 20->640, eval-mode U-Net, subtrees sharded over ranks",
                      "tiles": tiles, "last_level_batch": 256 // world if world <= 16 else None,
                      "gt_solve_s": round(gt_s, 3), "rmse_vs_gt640": m["rmse"], "mae_vs_gt640": m["mae"],
                      "tiles_per_s": round(tiles / (ms * 1e-3), 1),
                      "rel_err_vs_reference_output": ref_err}}
    if not args.no_cpu_baseline and world == 1:
        st = {k: v.detach().cpu() for k, v in model.state_dict().items()}
        rec["cpu_baseline"] = cpu_baseline_cascade(st, data, args.cpu_seconds)
    emit(rec)


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def measure_traffic_live(layer):
    """HBM bytes per launch of the roofline kernel, measured now on this build: two rocprofv3 PMC
    passes (FETCH_SIZE, WRITE_SIZE -- separate runs, --kernel-trace only) over tools/conv_bench.py
    running that layer's forward, reduced by tools/traffic_json.py (FETCH_SIZE x2, the guide's gfx950
    correction).  Child processes, each under a hard time limit, started before this process touches
    the GPU.  -> (bytes or None, source note)."""
    import shutil
    import subprocess
    import tempfile
    prof = shutil.which("rocprofv3")
    if prof is None:
        return None, "rocprofv3 not found"
    d = tempfile.mkdtemp(prefix="srpde_pmc_", dir="/tmp")
    env = dict(os.environ, TMPDIR="/tmp")
    exit_fault = None
    try:
        for i, c in enumerate(("FETCH_SIZE", "WRITE_SIZE")):
            cmd = ["timeout", "-s", "KILL", "90", prof, "--pmc", c, "--kernel-trace", "--output-format", "csv",
                   "-d", d, "-o", f"p{i}", "--", sys.executable, os.path.join(ROOT, "tools", "conv_bench.py"),
                   "--layers", layer, "--only", "fwd", "--iters", "3"]
            r = subprocess.run(cmd, cwd="/tmp", env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
            if r.returncode != 0:
                return None, f"PMC pass {c} failed (rc {r.returncode})"
        r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "traffic_json.py"), d, layer],
                           capture_output=True, text=True, timeout=120)
        rec = json.loads(r.stdout.strip().splitlines()[-1])
        val = rec.get(f"h3:{layer}")
        det = rec.get(f"h3:{layer}_detail", {})
        return (val if val else None,
                f"measured by this run: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE over tools/conv_bench.py {layer} fwd "
                f"(read {det.get('read_bytes')} B x2-corrected, written {det.get('write_bytes')} B per launch)")
    except Exception as e:   # noqa: BLE001 -- the bench line must not depend on the profiler
        return None, f"PMC measurement failed: {e}"
    finally:
        shutil.rmtree(d, ignore_errors=True)


def measure_step_traffic(batch):
    """HBM bytes per dispatch of every kernel of the training step, measured now on this build: two rocprofv3
    PMC passes (FETCH_SIZE, WRITE_SIZE -- separate runs, --kernel-trace only) over tools/step_once.py (the same
    step as the timed region), reduced by tools/kernel_traffic.py (FETCH_SIZE x2, the guide's gfx950
    correction).  Child processes under hard time limits, started before this process touches the GPU.
    -> ({kernel name: record} or None, source note)."""
    import shutil
    import subprocess
    import tempfile
    prof = shutil.which("rocprofv3")
    if prof is None:
        return None, "rocprofv3 not found"
    d = tempfile.mkdtemp(prefix="srpde_pmcs_", dir="/tmp")
    env = dict(os.environ, TMPDIR="/tmp")
    try:
        for i, c in enumerate(("FETCH_SIZE", "WRITE_SIZE")):
            cmd = ["timeout", "-s", "KILL", "150", prof, "--pmc", c, "--kernel-trace", "--output-format", "csv",
                   "-d", d, "-o", f"s{i}", "--", sys.executable, os.path.join(ROOT, "tools", "step_once.py"),
                   "--steps", "1", "--batch", str(batch)]
            r = subprocess.run(cmd, cwd="/tmp", env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
            if r.returncode != 0:
                return None, f"PMC pass {c} failed (rc {r.returncode})"
        r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "kernel_traffic.py"), d],
                           capture_output=True, text=True, timeout=120)
        return (json.loads(r.stdout.strip().splitlines()[-1]),
                "measured by this run: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) over "
                "tools/step_once.py (one warm-up + one training step), FETCH_SIZE x2 + WRITE_SIZE per dispatch, "
                "averaged over the kernel's dispatches (tools/kernel_traffic.py)")
    except Exception as e:   # noqa: BLE001 -- the bench line must not depend on the profiler
        return None, f"PMC measurement failed: {e}"
    finally:
        shutil.rmtree(d, ignore_errors=True)


def launch_ranks(args):
    """``--gpus N > 1`` without a launcher: start ``torch.distributed.run`` with N ranks (one process
    per GPU) as a CHILD process -- this process has made no GPU call yet and makes none -- relay the
    rank-0 JSON line on stdout and exit with the child's status."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    proc = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, text=True)
    for line in proc.stdout.splitlines():
        if line.lstrip().startswith("{"):
            print(line, flush=True)
    return proc.returncode


def main():
    global _JSON_OUT
    args = parse()
    args.ddp = args.ddp or args.ddp_rccl
    if os.environ.get("SRPDE_DUMP_MAPS"):
        # debug aid: this process's memory map at Python exit, to attribute the frames of a native crash in
        # a C-level exit handler (the rocprofv3 --pmc teardown fault)
        import atexit
        import shutil
        atexit.register(lambda: shutil.copyfile("/proc/self/maps", os.environ["SRPDE_DUMP_MAPS"]))
    ws = os.environ.get("WORLD_SIZE")
    if ws is None and args.gpus > 1:
        sys.exit(launch_ranks(args))
    if ws is not None and int(ws) != args.gpus and not (args.gpus == 1 and args.ddp):
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={ws} (launch one rank per GPU)", file=sys.stderr)
        sys.exit(2)
    live_traffic = None
    if (ws is None and args.workload == "train" and not args.no_live_traffic and args.traffic_json is None
            and not args.ddp):
        live_traffic = measure_traffic_live(args.roofline_layer)   # before this process touches the GPU
    step_traffic = (None, "not measured (--no-live-traffic / N > 1)")
    if ws is None and args.workload == "train" and not args.no_live_traffic and not args.ddp:
        step_traffic = measure_step_traffic(args.batch)
    pmc_poisson = None
    if ws is None and args.workload == "poisson" and not args.no_live_traffic:
        sz = args.poisson_sizes.split(",")
        head = [s for s in sz if int(s.split(":")[0]) <= 128]
        # the headline LDS CG and the largest grid-CG size: a counter run that makes a cooperative launch
        # faults in the HSA runtime's exit-time teardown AFTER rocprofv3 wrote its counters (frames
        # attributed to libhsa-runtime64 under libamdhip64's exit handler, profiles/r05b_pmc_exit.txt);
        # measure_traffic_poisson keeps the counters of such a pass
        grid = [s for s in sz if int(s.split(":")[0]) > 128]
        if head:
            pick = [next((s for s in head if s.startswith("80:")), head[0])] + grid[-1:]
            pmc_poisson = measure_traffic_poisson(",".join(pick))
    # RCCL prints its version block on fd 1 at communicator creation: keep fd 1 for the JSON line
    sys.stdout.flush()
    _JSON_OUT = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_pg = world > 1 or args.ddp
    if use_pg:
        # keep stdout to the one JSON line: RCCL's version banner is printed at the
        # VERSION debug level, so default the level to WARN unless the caller chose one
        os.environ.setdefault("NCCL_DEBUG", "WARN")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(world))
        # SRPDE_BENCH_BACKEND=gloo: rehearse the N > 1 path with several ranks on one GPU (RCCL
        # refuses two ranks on one device); the driver's runs use RCCL ("nccl")
        backend = os.environ.get("SRPDE_BENCH_BACKEND", "nccl")
        if backend != "nccl":
            local = local % torch.cuda.device_count()
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    if args.workload != "train":
        if args.workload == "poisson":
            run_poisson(args, world, rank, dev, pmc_poisson)
        else:
            run_cascade(args, world, rank, dev)
        if use_pg:
            dist.destroy_process_group()
        return

    from superresolution_for_pdes_amd.models import UNet, init_weights
    from superresolution_for_pdes_amd.functional import mse_loss
    from superresolution_for_pdes_amd.optim import FusedAdamW
    from superresolution_for_pdes_amd import unet_exec as X

    torch.manual_seed(42)
    model = UNet()
    model.apply(init_weights)
    model = model.to(dev).train()
    model.flatten_parameters_()
    net = model
    if use_pg:
        from superresolution_for_pdes_amd.distributed import DataParallel
        net = DataParallel(model, reduce_single_rank=args.ddp_rccl)
    opt = FusedAdamW(model.parameters(), lr=2e-4, weight_decay=1e-4, max_grad_norm=1.0)

    B = args.batch
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    x = torch.randn(B, 3, 40, 40, device=dev, generator=g)
    x[:, 1] = 1.0
    tgt = torch.randn(B, 1, 40, 40, device=dev, generator=g)

    def step():
        for p in model.parameters():
            p.grad = None
        out = net(x)
        loss = mse_loss(out, tgt)
        loss.backward()
        opt.step()
        return loss

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    # timed region: exactly K steps between barrier+sync pairs; roofline-layer conv
    # launches are bracketed with HIP events on the compute stream (the stream they run on)
    timed = []
    X.TIMED_LAYERS[args.roofline_layer] = timed
    # every conv launch of the timed region is bracketed with HIP events on its stream and labelled with the
    # kernel it ran (hipops.LAUNCH_TAP, srpde_last_kernel): the roofline prices the kernel with the largest
    # total time
    from superresolution_for_pdes_amd import hipops as H
    launches = []
    H.LAUNCH_TAP = launches
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    H.LAUNCH_TAP = None
    X.TIMED_LAYERS.pop(args.roofline_layer, None)
    if world > 1:
        tt = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt)
    # after the timed region: the forward alone (every rank runs it; rank 0 reports)
    math = H.conv_math()
    # dense MFMA peak of the instruction the kernel runs, in fp32-product units: fp32 MFMA
    # 157.3 TF; bf16 / fp16 MFMA run at 16x that (2516.8 TF), divided by the partial
    # products per fp32 product: 3 for h3 (838.9 TF)
    peak = {"h3": round(157.3 * 16 / 3, 1)}.get(math, 157.3)
    fwd_roof = forward_roofline(model, x, peak)

    if rank == 0:
        kern_ms = [a.elapsed_time(b) for a, b, _ in timed]
        kern_avg = sum(kern_ms) / max(len(kern_ms), 1)
        cin, cout, hw = next((c, o, h) for n, c, o, h in CONV3 if n == args.roofline_layer)
        flops_launch = conv_flops(cin, cout, hw) * B
        achieved = flops_launch / (kern_avg * 1e-3) / 1e12 if kern_avg > 0 else None
        kname = timed[0][2] if timed else {"h3": "conv_fwd_h3"}.get(math, "conv_fwd_v2")
        # per kernel over the timed region: launches, total ms (event pairs on the launching stream: the main
        # kernel plus the entry's small fixup / slab-reduction launches), algorithmic FLOP of its calls
        fam = {}
        for kn, fl, a, b in launches:
            r = fam.setdefault(kn, [0, 0.0, 0.0])
            r[0] += 1
            r[1] += a.elapsed_time(b)
            r[2] += fl
        table = sorted(fam.items(), key=lambda kv: -kv[1][1])
        top_name, (top_n, top_ms, top_fl) = table[0]
        top_ach = top_fl / (top_ms * 1e-3) / 1e12
        traffic, tfile, tsource = None, args.traffic_json or default_traffic_json(), None
        if live_traffic is not None and live_traffic[0] and math == "h3":
            traffic, tsource = live_traffic
        elif tfile and os.path.exists(tfile):
            try:
                traffic = json.load(open(tfile)).get(f"{math}:{args.roofline_layer}")
            except (ValueError, OSError):
                traffic = None
            if traffic:
                tsource = (os.path.relpath(tfile, ROOT) + " (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE per launch, "
                           "tools/gpu/round_evidence.sh)" +
                           (f"; live measurement unavailable: {live_traffic[1]}" if live_traffic else ""))
        samples = world * B * args.steps
        # whole-step fraction: algorithmic FLOP of every 3x3 conv pass the step runs (forward,
        # dgrad except enc1.conv1's, whose input needs no gradient, and wgrad) at batch B, over the
        # step time, against the same roof -- BN / attention / pooling / optimizer time included
        step_flop = sum(conv_flops(c, o, h) * B * (3 if n != "enc1.conv1" else 2) for n, c, o, h in CONV3)
        step_ach = step_flop / (elapsed / args.steps) / 1e12
        rec = {
            "metric": "20->40 SR training samples/sec at batch 1024 per GPU (fwd+MSE bwd+clip+AdamW)",
            "value": round(samples / elapsed, 2),
            "unit": "samples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": {"h3": "f32 (h3: fp32 products from power-of-two-scaled 2-piece fp16 splits on fp16 MFMA, "
                            "fp32 accumulate)"}.get(math, "f32"),
            "data": "synthetic (x~N(0,1), theta channel=1, t~N(0,1)), resident in HBM",
            "config": {"workload": "UNet 20->40 train step, fp32, batch 1024/GPU, 40x40",
                       "global_batch": world * B, "per_gpu_batch": B, "hw": "40x40",
                       "parallelism": f"dp{world}", "final_loss": round(float(loss.detach()), 6)},
            "roofline": {"bound": "mfma",
                         "kernel": top_name,
                         "kernel_note": "the conv kernel with the largest total time in the timed region (HIP events "
                                        "around every conv entry call on its stream, kernel names from "
                                        "srpde_last_kernel); achieved = the algorithmic FLOP of its calls / their time",
                         "achieved": round(top_ach, 2), "peak": peak, "unit": "TFLOP/s",
                         "frac": round(top_ach / peak, 4),
                         "launch_ms": round(top_ms / top_n, 4),
                         "launches": top_n, "algorithmic_flop": top_fl,
                         "traffic": ((step_traffic[0] or {}).get(top_name) or {}).get("bytes_per_dispatch"),
                         "traffic_source": step_traffic[1],
                         "traffic_detail": (step_traffic[0] or {}).get(top_name),
                         "kernels": [{"kernel": k, "launches": v[0], "ms": round(v[1], 3),
                                      "tflops": round(v[2] / (v[1] * 1e-3) / 1e12, 1),
                                      "frac": round(v[2] / (v[1] * 1e-3) / 1e12 / peak, 4)} for k, v in table[:12]],
                         "layer": {"kernel": f"{kname}[{args.roofline_layer}]",
                                   "achieved": round(achieved, 2) if achieved else None,
                                   "frac": round(achieved / peak, 4) if achieved else None,
                                   "launch_ms": round(kern_avg, 4), "algorithmic_flop_per_launch": flops_launch,
                                   "traffic": traffic, "traffic_source": tsource},
                         "step": {"algorithmic_flop": step_flop, "achieved": round(step_ach, 2),
                                  "frac": round(step_ach / peak, 4)},
                         "forward": fwd_roof},
        }
        if not args.no_cpu_baseline and world == 1:
            rec["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
        emit(rec)
    if use_pg:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
