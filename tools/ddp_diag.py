import os, sys, json, torch, torch.distributed as dist
sys.path.insert(0, os.environ["GRAFT_REPO_ROOT"])
rank = int(os.environ["RANK"]); dev = torch.device("cuda", 0); torch.cuda.set_device(dev)
dist.init_process_group("gloo")
from superresolution_for_pdes_amd.functional import mse_loss
from superresolution_for_pdes_amd.models import UNet, init_weights
torch.manual_seed(42); m = UNet(); m.apply(init_weights); m = m.to(dev).train(); m.flatten_parameters_()
g = torch.Generator(device=dev).manual_seed(1000 + rank)
x = torch.randn(64, 3, 40, 40, device=dev, generator=g); x[:, 1] = 1.0
t = torch.randn(64, 1, 40, 40, device=dev, generator=g)
res = []
for k in range(4):
    for p in m.parameters(): p.grad = None
    out = m(x); mse_loss(out, t).backward(); torch.cuda.synchronize()
    res.append((out.detach().cpu().clone(), torch.cat([p.grad.reshape(-1) for p in m.parameters()]).cpu()))
names = [n for n, _ in m.named_parameters()]
offs = []; o = 0
for _, p in m.named_parameters(): offs.append((o, p.numel())); o += p.numel()
for k in range(1, 4):
    do = float((res[k][0] - res[0][0]).abs().max()); dg = float((res[k][1] - res[0][1]).norm() / res[0][1].norm())
    bad = [names[i] for i, (a, n) in enumerate(offs) if not torch.equal(res[k][1][a:a+n], res[0][1][a:a+n])]
    print(f"rank {rank} step {k}: out maxdiff {do:.3e} grad rel {dg:.3e} differing {len(bad)}: {bad[:6]}", flush=True)
dist.barrier(); dist.destroy_process_group()
