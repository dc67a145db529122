"""Per-kernel table of the training step's HBM-bound backward kernels (verdict r5 item 2): for each dispatch of
bn_bwd_apply_split, bn_bwd_reduce, bn_bwd_apply, outer_sum, wgrad_reduce, slab_group_sum, upsample_bwd, att_bwd_*
and maxpool2_bwd in ONE B = 1024 training step: the algorithmic bytes (from the call's shapes), the PMC bytes
(FETCH_SIZE x 2 + WRITE_SIZE, MI355X_MICROARCH.md's gfx950 correction), and the fraction of 8 TB/s both inside the
step (the side stream's weight gradients running beside it) and alone (the same call re-issued right after with the
GPU otherwise idle).

    GPU:  python tools/membound_table.py run OUT_JSON          (under rocprofv3 --kernel-trace, and once per --pmc
                                                               counter; see tools/gpu/membound.sh)
    CPU:  python tools/membound_table.py table CALLS_JSON TRACE_DIR PMC_DIR... > profiles/r06_membound.md

The run mode patches hipops.call: phase A is a plain training step bracketed by two marker launches
(srpde_bn_eval_prepare on a 1-element tensor, a kernel the training step never runs); in phase B (the next step)
every HBM-bound call is issued, synchronised, then issued again between two markers -- the re-issue is the
"alone" dispatch.  Kernels are matched to calls per kernel name in launch order.
"""
import collections
import csv
import glob
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
HBM = 8.0e12


def cp32(c):
    return (c + 31) // 32 * 32


def expect(name, a):
    """-> [(kernel key, algorithmic bytes, shape label)] for one C entry call (args ``a``)."""
    if name == "srpde_bn_bwd_apply_split":
        P, C = a[10], a[11]
        return [("bn_bwd_apply_split_kernel", P * C * 8 + P * cp32(C) * 4, f"P={P} C={C}")]
    if name == "srpde_bn_bwd_prepare":
        P, C, part = a[8], a[9], a[11]
        return [] if part else [("bn_bwd_reduce_kernel", P * C * 8, f"P={P} C={C}")]
    if name in ("srpde_bn_relu_bwd", "srpde_bn_relu_bwd_part"):
        P, C = a[13], a[14]
        out = [("bn_bwd_reduce_kernel", P * C * 8, f"P={P} C={C}")] if name == "srpde_bn_relu_bwd" else []
        return out + [("bn_bwd_apply_kernel", P * C * 12, f"P={P} C={C}")]
    if name == "srpde_upsample_bilinear_bwd_gated":
        n, h, w, ho, wo, c, acc = a[6:13]
        return [("upsample_bwd", n * ho * wo * (c + 1) * 4 + n * h * w * c * 4 * (2 if acc else 1),
                 f"{h}->{ho} C={c} gated")]
    if name == "srpde_upsample_bilinear_bwd_gated_bn":   # + the BN backward reduction of dx (reads y)
        n, h, w, ho, wo, c = a[6:12]
        return [("upsample_bwd", n * ho * wo * (c + 1) * 4 + n * h * w * c * 8, f"{h}->{ho} C={c} gated+bn")]
    if name == "srpde_gating_bn_reduce":
        P, C = a[10], a[11]
        return [("gating_bn_reduce_kernel", P * C * 12 + P * 4, f"P={P} C={C}")]
    if name == "srpde_att_bwd_params_lowres":
        n, h, w, ho, wo, c, gc = a[2:9]
        Plo = n * h * w
        return (_att_params(n, h * w, c, gc)[:4]
                + [("upsample_t_scalar_kernel", n * ho * wo * 4 + Plo * 4, f"{ho}->{h} n={n}"),
                   ("weighted_colsum_kernel", Plo * gc * 4 + Plo * 4, f"P={Plo} gc={gc} low-res")])
    if name == "srpde_upsample_bilinear_bwd":
        n, h, w, ho, wo, c, acc = a[4:11]
        return [("upsample_bwd", n * ho * wo * c * 4 + n * h * w * c * 4 * (2 if acc else 1), f"{h}->{ho} C={c}")]
    if name == "srpde_maxpool2x2_bwd":
        n, h, w, c, acc = a[6:11]
        P = n * h * w
        return [("maxpool2_bwd", P * c * 4 + P // 4 * c * 4 + P * c * 4 * (2 if acc else 1), f"{h}x{w} C={c}")]
    if name == "srpde_att_bwd":
        n, hw, c, gc = a[6:10]
        dx_acc, pdg, dg_acc = a[19], a[20], a[22]
        P = n * hw
        out = []
        if c in (64, 128, 256):
            out.append(("att_bwd_sample_kernel", P * c * 8 + P * 4, f"P={P} C={c}"))
        else:
            out += [("att_bwd_pixel_kernel", P * c * 8 + P * 4, f"P={P} C={c}"),
                    ("att_bwd_channel_kernel", P * c * 8 + P * 4, f"P={P} C={c}")]
        out.append(("att_bwd_dx_kernel", P * c * 4 + P * 4 + P * c * 4 * (2 if dx_acc else 1), f"P={P} C={c}"))
        if pdg:
            out.append(("att_bwd_gating_kernel", P * 4 + P * gc * 4 * (2 if dg_acc else 1), f"P={P} gc={gc}"))
        if a[23]:   # parameter gradients in the same call
            out += _att_params(n, hw, c, gc)
        return out
    if name == "srpde_att_bwd_params":
        n, hw, c, gc = a[2:6]
        return _att_params(n, hw, c, gc)
    if name in ("srpde_conv_wgrad_h3p", "srpde_conv_wgrad_h3x", "srpde_conv_wgrad", "srpde_conv_wgrad_h3",
                "srpde_conv_wgrad_bnb"):
        if name == "srpde_conv_wgrad_bnb":
            c0, c1, acc, n, h, w, cout, ks, ws = a[12], 0, a[16], a[17], a[18], a[19], a[20], a[21], a[24]
        elif name == "srpde_conv_wgrad_h3p":
            c0, c1, acc, n, h, w, cout, ks, ws = a[3], a[5], a[9], a[10], a[11], a[12], a[13], a[14], a[17]
        elif name == "srpde_conv_wgrad_h3x":
            c0, c1, acc, n, h, w, cout, ks, ws = a[4], a[10], a[16], a[17], a[18], a[19], a[20], a[21], a[24]
        elif name == "srpde_conv_wgrad_h3":
            c0, c1, acc, n, h, w, cout, ks, ws = a[5], a[9], a[14], a[15], a[16], a[17], a[18], a[19], a[22]
        else:
            c0, c1, acc, n, h, w, cout, ks, ws = a[3], a[6], a[10], a[11], a[12], a[13], a[14], a[15], a[18]
        total = cout * ks * ks * (c0 + c1)
        splits = max(1, ws // (4 * total))
        lab = f"{n}x{h}x{w} {c0 + c1}->{cout}"
        out = []
        if total < 65536 and splits >= 128:
            g = (splits + 31) // 32
            out.append(("slab_group_sum_kernel", splits * total * 4 + g * total * 4, lab + f" splits={splits}"))
            splits = g
        out.append(("wgrad_reduce_kernel", splits * total * 4 + total * 4 * (2 if acc else 1), lab + f" splits={splits}"))
        return out
    return []


def _att_params(n, hw, c, gc):
    cr = c // 8
    P = n * hw
    return [("outer_sum_kernel", n * (cr + c) * 4 + cr * c * 4, f"dW1 n={n} C={c}"),
            ("outer_sum_kernel", n * (cr + c) * 4 + cr * c * 4, f"dW2 n={n} C={c}"),
            ("outer_sum_kernel", n * cr * 4 + cr * 4, f"db1 n={n} C={c}"),
            ("outer_sum_kernel", n * c * 4 + c * 4, f"db2 n={n} C={c}"),
            ("weighted_colsum_kernel", P * gc * 4 + P * 4, f"P={P} gc={gc}")]


MEMBOUND = {"srpde_bn_bwd_apply_split", "srpde_bn_bwd_prepare", "srpde_bn_relu_bwd", "srpde_bn_relu_bwd_part",
            "srpde_upsample_bilinear_bwd_gated", "srpde_upsample_bilinear_bwd", "srpde_maxpool2x2_bwd",
            "srpde_att_bwd", "srpde_att_bwd_params", "srpde_conv_wgrad_h3p", "srpde_conv_wgrad_h3x",
            "srpde_conv_wgrad", "srpde_conv_wgrad_h3", "srpde_upsample_bilinear_bwd_gated_bn", "srpde_gating_bn_reduce",
            "srpde_att_bwd_params_lowres", "srpde_conv_wgrad_bnb"}
MARKER = "bn_eval_prepare_kernel"


def run(out_json):
    import torch
    from superresolution_for_pdes_amd import hipops as H
    from superresolution_for_pdes_amd.functional import mse_loss
    from superresolution_for_pdes_amd.models import UNet, init_weights
    from superresolution_for_pdes_amd.optim import FusedAdamW
    dev = torch.device("cuda", 0)
    torch.manual_seed(42)
    model = UNet()
    model.apply(init_weights)
    model = model.to(dev).train()
    model.flatten_parameters_()
    opt = FusedAdamW(model.parameters(), lr=2e-4, weight_decay=1e-4, max_grad_norm=1.0)
    g = torch.Generator(device=dev).manual_seed(1234)
    x = torch.randn(1024, 3, 40, 40, device=dev, generator=g)
    x[:, 1] = 1.0
    tgt = torch.randn(1024, 1, 40, 40, device=dev, generator=g)
    one = torch.ones(1, device=dev)

    def marker():
        H.bn_eval_prepare(one, one, 1e-5)

    def step():
        for p in model.parameters():
            p.grad = None
        loss = mse_loss(model(x), tgt)
        loss.backward()
        opt.step()

    for _ in range(2):
        step()
    torch.cuda.synchronize()
    orig = H.call
    calls = []
    mode = ["record"]

    def hooked(name, *args):
        rc = orig(name, *args)
        if name in MEMBOUND:
            if mode[0] == "record":
                calls.append({"name": name, "args": [int(v) if isinstance(v, int) else v for v in args],
                              "expect": expect(name, args)})
            elif mode[0] == "alone" and expect(name, args):
                torch.cuda.synchronize()
                marker()
                orig(name, *args)
                marker()
                torch.cuda.synchronize()
        return rc

    H.call = hooked
    marker()
    step()                       # phase A: the step as it runs
    torch.cuda.synchronize()
    marker()
    torch.cuda.synchronize()
    mode[0] = "alone"
    step()                       # phase B: every HBM-bound call re-issued alone
    torch.cuda.synchronize()
    H.call = orig
    json.dump([{"name": c["name"], "expect": c["expect"]} for c in calls], open(out_json, "w"))
    print(f"{len(calls)} calls recorded, {sum(len(c['expect']) for c in calls)} kernels expected")


def _norm(k):
    from kernel_traffic import norm
    return norm(k)


def _dispatches(d, fname):
    rows = []
    for f in glob.glob(f"{d}/**/*{fname}", recursive=True):
        rows += list(csv.DictReader(open(f)))
    return rows


def _phases(rows, key):
    """rows sorted by start -> (phase A rows, [alone groups]) split at the marker kernels"""
    rows = sorted(rows, key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if MARKER in r["Kernel_Name"]]
    a = rows[idx[0] + 1:idx[1]]
    groups = [rows[idx[i] + 1:idx[i + 1]] for i in range(2, len(idx) - 1, 2)]
    return a, groups


def table(calls_json, trace_dir, pmc_dirs):
    calls = json.load(open(calls_json))
    trace = _dispatches(trace_dir, "kernel_trace.csv")
    a_rows, groups = _phases(trace, None)
    # per call (only calls with expectations get an alone group, in call order)
    keyed = collections.defaultdict(list)   # kernel key -> phase-A dispatch rows in order
    exp_keys = {k for c in calls for k, _, _ in c["expect"]}
    for r in a_rows:
        n = _norm(r["Kernel_Name"])
        for k in exp_keys:
            if k in n:
                keyed[k].append(r)
    # PMC per dispatch (phase A, by kernel key in order; alone groups likewise)
    pmc = {}
    for d in pmc_dirs:
        rows = _dispatches(d, "counter_collection.csv")
        if not rows:
            continue
        cname = rows[0]["Counter_Name"]
        ra, rg = _phases(rows, None)
        kk = collections.defaultdict(list)
        for r in ra:
            n = _norm(r["Kernel_Name"])
            for k in exp_keys:
                if k in n:
                    kk[k].append(float(r["Counter_Value"]))
        pmc[cname] = (kk, rg)
    used = collections.defaultdict(int)
    out_rows = []
    gi = 0
    for c in calls:
        if not c["expect"]:
            continue
        grp = groups[gi] if gi < len(groups) else []
        gpmc = {cn: (rg[gi] if gi < len(rg) else []) for cn, (kk, rg) in pmc.items()}
        gi += 1
        gused = collections.defaultdict(int)
        for k, alg, lab in c["expect"]:
            i = used[k]
            used[k] += 1
            ra = keyed[k][i] if i < len(keyed[k]) else None
            t_step = (int(ra["End_Timestamp"]) - int(ra["Start_Timestamp"])) / 1e3 if ra else float("nan")
            cand = [r for r in grp if k in _norm(r["Kernel_Name"])]
            j = gused[k]
            gused[k] += 1
            rb = cand[j] if j < len(cand) else None
            t_alone = (int(rb["End_Timestamp"]) - int(rb["Start_Timestamp"])) / 1e3 if rb else float("nan")
            pb = None
            if "FETCH_SIZE" in pmc and "WRITE_SIZE" in pmc:
                fa, wa = pmc["FETCH_SIZE"][0][k], pmc["WRITE_SIZE"][0][k]
                if i < len(fa) and i < len(wa):
                    pb = 2 * 1024 * fa[i] + 1024 * wa[i]
            out_rows.append({"kernel": k, "call": c["name"], "shape": lab, "alg_bytes": alg, "us_step": t_step,
                             "us_alone": t_alone, "pmc_bytes": pb})
    print("| kernel | shape | alg MB | PMC MB | PMC / alg | in step µs | TB/s in step | frac of 8 TB/s | alone µs | "
          "TB/s alone | frac alone |")
    print("|---|---|---|---|---|---|---|---|---|---|---|")
    tot = collections.defaultdict(lambda: [0, 0.0, 0.0, 0.0])
    for r in out_rows:
        alg = r["alg_bytes"]
        ts, tl = r["us_step"], r["us_alone"]
        bw_s = alg / ts / 1e6 if ts == ts and ts > 0 else float("nan")
        bw_l = alg / tl / 1e6 if tl == tl and tl > 0 else float("nan")
        pb = r["pmc_bytes"]
        print(f"| {r['kernel']} | {r['shape']} | {alg / 1e6:.1f} | {'' if pb is None else f'{pb / 1e6:.1f}'} | "
              f"{'' if pb is None else f'{pb / alg:.2f}'} | {ts:.1f} | {bw_s:.2f} | {bw_s * 1e12 / HBM:.3f} | "
              f"{tl:.1f} | {bw_l:.2f} | {bw_l * 1e12 / HBM:.3f} |")
        t = tot[r["kernel"]]
        t[0] += 1
        t[1] += alg
        t[2] += ts if ts == ts else 0
        t[3] += tl if tl == tl else 0
    print()
    print("| kernel | calls / step | alg GB / step | ms / step in step | ms alone | frac in step | frac alone |")
    print("|---|---|---|---|---|---|---|")
    for k, (n, alg, ts, tl) in sorted(tot.items(), key=lambda kv: -kv[1][2]):
        print(f"| {k} | {n} | {alg / 1e9:.3f} | {ts / 1e3:.3f} | {tl / 1e3:.3f} | "
              f"{alg / (ts * 1e-6) / HBM if ts else 0:.3f} | {alg / (tl * 1e-6) / HBM if tl else 0:.3f} |")
    json.dump(out_rows, open(calls_json.replace(".json", "_rows.json"), "w"), indent=0)


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2])
    else:
        table(sys.argv[2], sys.argv[3], sys.argv[4:])
