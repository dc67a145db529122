"""One rank of the world-2 DataParallel U-Net step check (tests/test_gpu_ddp.py launches two of
these with torch.distributed.run; both ranks share the one GPU, so the group is gloo -- RCCL refuses
two ranks on one device; the reducer, its side stream and the executor are the RCCL path's).

Per rank: the single-process gradient of its own shard (no reducer), then the DataParallel step on
the same shard (bucketed all-reduce overlapped with the backward), then FusedAdamW.  Rank 0 writes
a JSON verdict to argv[1].  Reference loop sharded: src/train_enhanced.py:65-77."""
import json
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    out_path = sys.argv[1]
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo")
    from superresolution_for_pdes_amd.distributed import DataParallel
    from superresolution_for_pdes_amd.functional import mse_loss
    from superresolution_for_pdes_amd.models import UNet, init_weights
    from superresolution_for_pdes_amd.optim import FusedAdamW

    torch.manual_seed(42)
    model = UNet()
    model.apply(init_weights)
    model = model.to(dev).train()
    model.flatten_parameters_()
    g = torch.Generator(device=dev).manual_seed(1000 + rank)
    x = torch.randn(B, 3, 40, 40, device=dev, generator=g)
    x[:, 1] = 1.0
    t = torch.randn(B, 1, 40, 40, device=dev, generator=g)
    bufs0 = [b.detach().clone() for b in model.buffers()]

    # 1. this rank's single-process gradient (no reducer attached yet)
    for p in model.parameters():
        p.grad = None
    mse_loss(model(x), t).backward()
    torch.cuda.synchronize()
    flat_of = lambda: torch.cat([p.grad.reshape(-1) for p in model.parameters()]).cpu()  # noqa: E731
    local = flat_of()
    parts = [torch.empty_like(local) for _ in range(world)]
    dist.all_gather(parts, local)
    want = sum(parts) / world
    with torch.no_grad():                        # undo the running-statistic update of step 1
        for b, b0 in zip(model.buffers(), bufs0):
            b.copy_(b0)
        if rank == 1:                            # DataParallel must overwrite a diverged replica
            for name, b in model.named_buffers():
                if name.endswith("running_mean"):
                    b.add_(1.0)

    # 2. the DataParallel step on the same shard
    net = DataParallel(model)
    opt = FusedAdamW(model.parameters(), lr=2e-4, weight_decay=1e-4, max_grad_norm=1.0)
    for p in model.parameters():
        p.grad = None
    out = net(x)
    nbt = torch.stack([b for n, b in model.named_buffers() if n.endswith("num_batches_tracked")]).cpu()
    mse_loss(out, t).backward()
    torch.cuda.synchronize()
    red = flat_of()
    rel = float((red - want).norm() / want.norm())
    per_tensor = max(float((red[o:o + n] - want[o:o + n]).norm() / max(want[o:o + n].norm(), 1e-30))
                     for o, n in _offsets(model))
    # BN buffers: rank 0's broadcast before the forward (num_batches_tracked = rank 0's + 1), and
    # after sync_buffers every rank holds rank 0's statistics
    nbt_all = [torch.empty_like(nbt) for _ in range(world)]
    dist.all_gather(nbt_all, nbt)
    net.sync_buffers()
    bflat = torch.cat([b.double().reshape(-1) for b in model.buffers()]).cpu()
    ball = [torch.empty_like(bflat) for _ in range(world)]
    dist.all_gather(ball, bflat)
    # 3. the optimizer: identical parameters on every rank afterwards
    opt.step()
    torch.cuda.synchronize()
    pflat = torch.cat([p.detach().reshape(-1) for p in model.parameters()]).cpu()
    pall = [torch.empty_like(pflat) for _ in range(world)]
    dist.all_gather(pall, pflat)
    if rank == 0:
        rec = {"world": world, "batch_per_rank": B, "grad_rel": rel, "grad_rel_max_tensor": per_tensor,
               "ranks_differ": float((parts[0] - parts[1]).norm() / parts[0].norm()),
               "nbt_equal": all(torch.equal(v, nbt_all[0]) for v in nbt_all),
               "buffers_equal": all(torch.equal(v, ball[0]) for v in ball),
               "params_equal": all(torch.equal(v, pall[0]) for v in pall),
               "n_buckets": model._grad_reducer.n_buckets}
        with open(out_path, "w") as f:
            json.dump(rec, f)
    dist.barrier()
    dist.destroy_process_group()


def _offsets(model):
    off = 0
    for p in model.parameters():
        yield off, p.numel()
        off += p.numel()


if __name__ == "__main__":
    main()
