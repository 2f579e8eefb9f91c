"""Data-parallel fine-tune: the DistributedDataParallel drop-in over RCCL.

Reference: semantic_seg_multigpu.py:467-468 (init_process_group), :511 (DDP(model,
device_ids=[gpu])), rmbsnn_main.py:223 — one process per GPU, gradients averaged across ranks
by DDP's bucketed all-reduce overlapped with backward, BN buffers broadcast from rank 0 before
every forward (DDP's broadcast_buffers=True default), no SyncBN.

MI355X design:
  * The train-mode DRNSeg backward (drnmi.train.TrainRunner) writes every parameter's .grad
    into ONE flat fp32 buffer laid out in backward order, so an all-reduce bucket is a plain
    contiguous slice — no pack/unpack copies around the collective.
  * The runner calls back after each node's weight/BN gradients land; a bucket whose
    parameters are all ready is handed to `dist.all_reduce(..., async_op=True)` at once, so
    RCCL moves bucket b over xGMI while the HIP kernels of earlier layers are still running
    (the "nccl" backend is RCCL on ROCm; it orders itself after the current stream).
  * Averaging costs nothing: the runner scales dL/dlogprobs by 1/world_size at the head (every
    gradient is linear in it; for power-of-two world sizes the scaling is exact), so the
    all-reduce is a plain SUM.
  * Default bucket 25 MB (DDP's default) — D-22's 63.6 MB of gradients go in 3 buckets, D-54's
    141 MB in 6; on 8 ranks a ring all-reduce moves 2*(N-1)/N of a bucket per link.
The bucket logic (BucketReducer) is device-agnostic and covered by a gloo world-2 CPU test.
"""
from __future__ import annotations

import torch
import torch.distributed as dist
import torch.nn as nn


class BucketReducer:
    """Launches an async SUM all-reduce of each contiguous bucket of `flat` as soon as all of
    its parameters are reported ready; `finalize()` waits for all of them."""

    def __init__(self, flat: torch.Tensor, params, bucket_cap_bytes: int = 25 << 20, group=None):
        self.flat = flat
        self.group = group
        self.buckets = []          # (start, end, frozenset(param ids))
        self.bucket_of = {}
        start, ids, size = 0, [], 0
        off = 0
        for p in params:
            n = p.numel()
            ids.append(id(p))
            size += n * flat.element_size()
            off += n
            if size >= bucket_cap_bytes:
                self._close(start, off, ids)
                start, ids, size = off, [], 0
        if ids:
            self._close(start, off, ids)
        self.reset()

    def _close(self, start, end, ids):
        b = len(self.buckets)
        self.buckets.append((start, end, frozenset(ids)))
        for i in ids:
            self.bucket_of[i] = b

    def reset(self):
        """Start a step with no bucket launched.  A bucket collective still in flight (a backward
        that raised part-way left it launched) is waited for first, so it cannot keep writing into
        the flat gradient buffer while the next backward fills it."""
        for h in getattr(self, "handles", ()):
            if h is not None:
                h.wait()
        self.pending = [set(ids) for _, _, ids in self.buckets]
        self.handles = [None] * len(self.buckets)
        self.launch_order = []

    def mark_ready(self, params):
        for p in params:
            b = self.bucket_of.get(id(p))
            if b is None:
                continue
            self.pending[b].discard(id(p))
            if not self.pending[b] and self.handles[b] is None:
                s, e, _ = self.buckets[b]
                self.handles[b] = dist.all_reduce(self.flat[s:e], op=dist.ReduceOp.SUM, group=self.group,
                                                  async_op=True)
                self.launch_order.append(b)

    def finalize(self):
        for b, h in enumerate(self.handles):
            if h is None:      # parameters that got no gradient this step: reduce the bucket anyway
                s, e, _ = self.buckets[b]
                h = dist.all_reduce(self.flat[s:e], op=dist.ReduceOp.SUM, group=self.group, async_op=True)
                self.launch_order.append(b)
            h.wait()
            self.handles[b] = None
        self.reset()


class DistributedDataParallel(nn.Module):
    """torch.nn.parallel.DistributedDataParallel drop-in for drnmi.DRNSeg fine-tuning.

    Usage mirrors the reference (semantic_seg_multigpu.py:511):
        model = DistributedDataParallel(DRNSeg(...).cuda(), device_ids=[local_rank])
        output = model(input)[0]; loss = criterion(output, target)
        optimizer.zero_grad(); loss.backward(); optimizer.step()
    state_dict keys gain the usual "module." prefix (the pruners resolve both forms)."""

    def __init__(self, module, device_ids=None, bucket_cap_mb: float = 25, broadcast_buffers: bool = True,
                 process_group=None):
        super().__init__()
        if not (dist.is_available() and dist.is_initialized()):
            raise RuntimeError("DistributedDataParallel needs torch.distributed.init_process_group first")
        self.module = module
        self.group = process_group
        self.world = dist.get_world_size(process_group)
        self.broadcast_buffers = broadcast_buffers
        self.bucket_cap = int(bucket_cap_mb * (1 << 20))
        self._reducer = None
        self._queued = False
        from .train import TrainRunner
        runner = getattr(module, "_train_runner", None)
        if runner is None:
            runner = TrainRunner(module)
            module._train_runner = runner
        self.runner = runner
        runner.grad_scale = 1.0 / self.world
        runner.grad_ready = self._grad_ready
        self._sync_module_states()

    def _sync_module_states(self):
        """Rank 0's parameters and buffers everywhere (DDP's constructor broadcast)."""
        with torch.no_grad():
            for t in list(self.module.parameters()) + list(self.module.buffers()):
                dist.broadcast(t.detach(), 0, group=self.group)
                torch.autograd.graph.increment_version(t)   # eval plans repack on version change

    def forward(self, *args, **kwargs):
        # a backward that raised part-way never ran _finalize: start every step from a clean
        # reducer (reset waits for any bucket collective still in flight).  This keeps the local
        # buffers consistent; it cannot repair a rank that skipped collectives its peers issued --
        # such a job hangs in the peers' next collective, as torch DDP does
        self._queued = False
        if self._reducer is not None:
            self._reducer.reset()
        if self.broadcast_buffers and self.module.training and self.world > 1:
            with torch.no_grad():
                for b in self.module.buffers():
                    dist.broadcast(b, 0, group=self.group)
                    torch.autograd.graph.increment_version(b)
        return self.module(*args, **kwargs)

    def _grad_ready(self, params):
        r = self.runner
        if self._reducer is None or self._reducer.flat is not r._flat:
            self._reducer = BucketReducer(r._flat, r._flat_params, self.bucket_cap, self.group)
        if not self._queued:
            self._queued = True
            torch.autograd.Variable._execution_engine.queue_callback(self._finalize)
        self._reducer.mark_ready(params)

    def _finalize(self):
        self._queued = False
        try:
            self._reducer.finalize()
        finally:
            self._reducer.reset()

    # the reference calls these on the wrapped model
    def optim_parameters(self, memo=None):
        return self.module.optim_parameters(memo)

