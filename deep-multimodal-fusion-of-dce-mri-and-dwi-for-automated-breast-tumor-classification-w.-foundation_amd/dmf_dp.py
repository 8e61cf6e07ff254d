"""Data-parallel fusion training driver (one process per GPU, RCCL over xGMI).

Replaces the Lightning Trainer that ``run_training.run_fusion_model``
(run_training.py:181-333) builds, for the hot path only:
  * rank-strided sampling of volumes (each rank its own local batch; BN stays
    LOCAL, as the reference uses plain BatchNorm2d -- SURVEY.md 8(e));
  * ONE gradient exchange per step: the gradients of every trainable
    parameter are packed into a single fp32 bucket (one kernel), summed with
    one ``all_reduce`` (backend "nccl" == RCCL), and the AdamW kernel reads the
    reduced bucket directly with scale 1/world (no unpack pass);
  * the step (forward + backward + pack [+ all-reduce] + AdamW) is captured
    into hipGraphs after warm-up, so the Python launch overhead is paid once;
  * epoch-end AUROC over the all-gathered probabilities (metrics.py).
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def dist_env():
    """(rank, local_rank, world) from the torchrun environment (1-process defaults)."""
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("LOCAL_RANK", 0)),
            int(os.environ.get("WORLD_SIZE", 1)))


def rank_strided_indices(n_items, rank, world, epoch=0, shuffle=False, seed=0):
    """Disjoint per-rank index lists (DistributedSampler semantics, padded by
    wrap-around so every rank gets the same count). The reference's fusion
    loader never shuffles (quirk Q11), so shuffle defaults to False."""
    idx = list(range(n_items))
    if shuffle:
        g = torch.Generator().manual_seed(seed + epoch)
        idx = torch.randperm(n_items, generator=g).tolist()
    per = (n_items + world - 1) // world
    total = per * world
    pad = total - n_items
    if pad > 0 and idx:
        idx = idx + (idx * (pad // len(idx) + 1))[:pad]
    return idx[rank:total:world]


def allreduce_mean_(bucket, world, group=None):
    """Sum a flat bucket over ranks, in place; the 1/world factor is applied
    by the consumer (AdamW grad_scale) so the bucket is touched once."""
    if world > 1:
        dist.all_reduce(bucket, op=dist.ReduceOp.SUM, group=group)
    return bucket


def allgather_rows(t, world):
    """Concatenate a [n, ...] tensor from all ranks (equal n per rank)."""
    if world == 1:
        return t
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t.contiguous())
    return torch.cat(parts, 0)


class FusionTrainer:
    """Owns the LightningFusionModel-equivalent, its FusedAdamW and the
    captured step. ``step(batch)`` runs one training step."""

    def __init__(self, lm, world=1, use_graph=True):
        self.lm = lm
        self.world = world
        self.use_graph = use_graph
        cfg = lm.configure_optimizers()
        self.opt = cfg["optimizer"] if isinstance(cfg, dict) else cfg
        self.lm.optimizer = self.opt
        self.graphs = None
        self.static_batch = None
        self._bucket_ready = False
        self.loss = None

    # ---------------------------------------------------------- eager step
    def _fwd_bwd(self, batch):
        self.opt.zero_grad(set_to_none=False)
        loss = self.lm.training_step(batch)
        loss.backward()
        return loss

    def _exchange_and_update(self):
        if self.world > 1:
            self.opt.pack_grads()
            allreduce_mean_(self.opt.bucket, self.world)
        self.opt.step()

    def _setup_bucket(self):
        params = [p for g in self.opt.param_groups for p in g["params"] if p.grad is not None]
        if self.world > 1 and params:
            self.opt.make_bucket(params)
            self.opt.use_bucket_grads(True, 1.0 / self.world)
        self._bucket_ready = True

    def eager_step(self, batch):
        loss = self._fwd_bwd(batch)
        if not self._bucket_ready:
            self._setup_bucket()
        self._exchange_and_update()
        self.lm.global_step += 1
        self.loss = loss.detach()
        return loss

    # ----------------------------------------------------------- graphs
    def capture(self, batch):
        """Capture fwd+bwd(+pack) and the update as hipGraphs; the RCCL
        all-reduce between them stays eager (one collective per step)."""
        self.static_batch = tuple(t.clone() for t in batch)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):  # warm the allocator / tables on the side stream
                self.eager_step(self.static_batch)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        g1 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g1):
            self.loss = self._fwd_bwd(self.static_batch)
            if self.world > 1:
                self.opt.pack_grads()
        g2 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g2):
            self.opt.step()
        self.graphs = (g1, g2)

    def step(self, batch=None):
        if self.graphs is None:
            return self.eager_step(batch)
        if batch is not None and batch[0].data_ptr() != self.static_batch[0].data_ptr():
            for dst, src in zip(self.static_batch, batch):
                dst.copy_(src, non_blocking=True)
        g1, g2 = self.graphs
        g1.replay()
        if self.world > 1:
            allreduce_mean_(self.opt.bucket, self.world)
        g2.replay()
        self.lm.global_step += 1
        return self.loss
