"""Data-parallel training over RCCL (torch.distributed backend "nccl" == RCCL on ROCm).

New relative to the reference (which is single-process): one process per
GPU, each rank runs the HIP U-Net on its own minibatch shard, and the flat gradient
buffer is all-reduced in buckets *while the backward is still running*:

* the executor writes gradients into one flat buffer laid out in backward-completion
  order (unet_exec.FLAT_GROUPS), and calls ``ready(offset)`` whenever a module group's
  gradients are final -- a growing prefix;
* ``GradReducer`` records an event on the compute stream, makes its side stream wait on
  it (and on the executor's weight-gradient stream), and issues ``all_reduce`` of every finished ``bucket_bytes`` chunk on that side
  stream, so RCCL traffic over xGMI overlaps the remaining dgrad/wgrad kernels;
* ``finish()`` flushes the tail and makes the compute stream wait for the side stream.

Averaging uses ReduceOp.AVG on RCCL (SUM + scale on gloo, which lacks AVG), so the
gradients handed back to autograd are the global mean, exactly what a single process
with the concatenated batch would see for a sum-decomposable loss.  BatchNorm stays
per-rank (the reference has no SyncBN); running statistics are broadcast from rank 0
each step (``broadcast_buffers``), as torch DDP does by default.
"""
from __future__ import annotations

import contextlib

import torch
import torch.distributed as dist

_null = contextlib.nullcontext


class GradReducer:
    def __init__(self, process_group=None, bucket_bytes: int = 8 << 20):
        self.pg = process_group
        self.bucket = max(1, bucket_bytes // 4)
        self.world = dist.get_world_size(process_group)
        self.backend = dist.get_backend(process_group)
        self.use_avg = self.backend == "nccl"
        self.flat = None
        self.launched = 0
        self.works = []
        self.stream = None
        self.n_buckets = 0
        self.buckets = []
        self.wait_streams = ()

    def _side_stream(self, dev):
        if dev.type != "cuda":
            return None
        if self.stream is None or self.stream.device != dev:
            self.stream = torch.cuda.Stream(device=dev)
        return self.stream

    def begin(self, flat, wait_streams=()):
        """``wait_streams``: further streams that write the flat gradient (the executor's
        weight-gradient side stream); every bucket also waits for them."""
        self.flat = flat
        self.wait_streams = tuple(wait_streams)
        self.launched = 0
        self.works = []
        self.buckets = []
        self.n_buckets = 0

    # a one-rank group has nothing to reduce: the mean over one rank is the gradient itself.  RCCL still
    # runs its one-rank all-reduce as a scaled copy of every bucket (oneRankReduce, 31 MB in and out,
    # 0.2 ms of kernels beside the backward: +1.4 % on the world-1 step, profiles/r04l_dp_world1.txt).
    # DataParallel(reduce_single_rank=True) keeps it (the one-GPU rehearsal of the RCCL path).
    skip_single_rank = True

    def _collective(self, chunk):
        """Issue the bucket's all-reduce on the current stream; returns the async work (or None
        for a stream-ordered stand-in, see tests/test_gpu_schedule.py, or a one-rank group)."""
        if self.world == 1 and self.skip_single_rank:
            return None
        op = dist.ReduceOp.AVG if self.use_avg else dist.ReduceOp.SUM
        return dist.all_reduce(chunk, op=op, group=self.pg, async_op=True)

    def _launch(self, lo, hi):
        chunk = self.flat[lo:hi]
        st = self._side_stream(self.flat.device)
        self.buckets.append((lo, hi))
        if st is not None:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.flat.device))
            st.wait_event(ev)
            for s in self.wait_streams:
                st.wait_stream(s)
            with torch.cuda.stream(st):
                self.works.append((self._collective(chunk), chunk))
        else:
            self.works.append((self._collective(chunk), chunk))
        self.n_buckets += 1

    def ready(self, upto: int):
        while upto - self.launched >= self.bucket:
            self._launch(self.launched, self.launched + self.bucket)
            self.launched += self.bucket

    def finish(self):
        total = self.flat.numel()
        if self.launched < total:
            self._launch(self.launched, total)
            self.launched = total
        cur = torch.cuda.current_stream(self.flat.device) if self.flat.is_cuda else None
        for work, chunk in self.works:
            # the SUM -> mean division runs on the stream the collective's result is ordered on
            # (the side stream): on the compute stream it could overtake the copy-back
            with torch.cuda.stream(self.stream) if cur is not None else _null():
                if work is not None:
                    work.wait()
                if not self.use_avg:
                    chunk.div_(self.world)
        if cur is not None:
            cur.wait_stream(self.stream)
        self.works = []


class DataParallel(torch.nn.Module):
    """Wrap a UNet for one-process-per-GPU data parallelism (replaces nothing in the
    reference; see module docstring).  ``forward`` broadcasts BN buffers from rank 0 and
    runs the wrapped model; its backward all-reduces gradients bucket by bucket."""

    def __init__(self, module, process_group=None, bucket_bytes: int = 8 << 20, broadcast_buffers: bool = True,
                 reduce_single_rank: bool = False):
        """``reduce_single_rank``: run the buckets' all-reduce even in a one-rank group (RCCL's one-rank
        reduce, a scaled copy per bucket), so a one-GPU rehearsal carries RCCL's kernels and stream beside
        the backward exactly as an N > 1 step does; the default skips it (nothing to reduce)."""
        super().__init__()
        self.module = module
        self.pg = process_group
        self.broadcast_buffers = broadcast_buffers
        module._grad_reducer = GradReducer(process_group, bucket_bytes)
        module._grad_reducer.skip_single_rank = not reduce_single_rank
        self._sync_params()

    @torch.no_grad()
    def _sync_params(self):
        for p in self.module.parameters():
            dist.broadcast(p.data, 0, group=self.pg)
        self._sync_buffers()

    @torch.no_grad()
    def _sync_buffers(self):
        # one broadcast per dtype (fp32 running stats, int64 batch counters), multi-tensor copies
        by_dtype = {}
        for b in self.module.buffers():
            by_dtype.setdefault(b.dtype, []).append(b)
        for bufs in by_dtype.values():
            flat = torch.cat([b.reshape(-1) for b in bufs])
            dist.broadcast(flat, 0, group=self.pg)
            parts = torch.split(flat, [b.numel() for b in bufs])
            torch._foreach_copy_(bufs, [s.view_as(b) for s, b in zip(parts, bufs)])

    def sync_buffers(self):
        """Broadcast rank 0's BN buffers now (train_model calls it before validation, so every
        rank evaluates the model rank 0 checkpoints)."""
        if dist.get_world_size(self.pg) > 1:
            self._sync_buffers()

    def forward(self, x):
        if self.broadcast_buffers and self.module.training and dist.get_world_size(self.pg) > 1:
            buf = next(self.module.buffers(), None)
            if buf is not None and buf.is_cuda:
                # off the compute stream (verdict r3 #9): the broadcast runs on the reducer's side
                # stream after the previous step's writes of the buffers, and the executor makes the
                # compute stream wait for it only before the step's first BatchNorm finalize (the
                # first kernel that reads or writes a running statistic), so it overlaps the input
                # transpose and the first convolution
                from . import unet_exec
                cur = torch.cuda.current_stream(buf.device)
                st = self.module._grad_reducer._side_stream(buf.device)
                st.wait_stream(cur)
                with torch.cuda.stream(st):
                    self._sync_buffers()
                ev = torch.cuda.Event()
                ev.record(st)
                unet_exec.buffers_pending(ev)
            else:
                self._sync_buffers()
        return self.module(x)


def shard_indices(n: int, rank: int, world: int, seed: int, epoch: int = 0, shuffle: bool = True):
    """DistributedSampler semantics: a seeded permutation padded to a multiple of world,
    rank r takes elements r, r+world, ...  (every rank sees n_per_rank samples)."""
    g = torch.Generator().manual_seed(seed + epoch)
    idx = torch.randperm(n, generator=g) if shuffle else torch.arange(n)
    per = (n + world - 1) // world
    total = per * world
    if total > n:
        idx = torch.cat([idx, idx[: total - n]])
    return idx[rank:total:world]
