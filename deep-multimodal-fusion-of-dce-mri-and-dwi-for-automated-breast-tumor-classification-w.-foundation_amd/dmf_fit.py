"""Epoch driver of the data-parallel fusion training (one process per GPU).

The slice of the Lightning ``Trainer.fit`` loop that
``run_training.run_fusion_model`` drives (run_training.py:181-333) around the
hot path, without Lightning:

  * epoch start: ``current_epoch`` and the gradual-unfreeze hook
    (train_fusion.py:155-169, selector_helpers.py:541-613); a changed
    trainable set makes ``FusionTrainer`` re-capture its step;
  * training: this rank's strided shard of the training set
    (DistributedSampler semantics, padded by wrap-around so every rank runs
    the same number of steps), local batches of ``batch_size`` volumes, one
    captured ``FusionTrainer.step`` each (gradient all-reduce inside); an
    epoch's ragged last batch runs eagerly;
  * validation (train.py:654-695, train_fusion.py:342-405): eval mode, the
    ``_shared_step(.., "val")`` loss and softmax probabilities of every local
    batch; ``val_loss`` = the sample-weighted mean over the whole validation
    set (Lightning's ``on_epoch`` mean weighted by batch size), all-reduced;
    probabilities and labels all-gathered from every rank (padding rows
    dropped) into the macro one-vs-rest AUROC over the concatenated epoch
    (torchmetrics MulticlassAUROC, metrics.multiclass_auroc);
  * epoch end: ReduceLROnPlateau stepped with the all-reduced ``val_loss``
    (selector_helpers.py:148-156, monitor "val_loss"), so every rank holds
    the same learning rates.

Validation is exact under any world size: eval-mode BN and no dropout make
each volume's logits independent of its batch-mates, so the gathered AUROC
and the weighted val_loss equal the single-process ones.
"""
from __future__ import annotations

import math

import torch
import torch.distributed as dist

import metrics
from dmf_dp import FusionTrainer, rank_strided_indices


def shard(n_items, rank, world):
    """(items, valid) of this rank: DistributedSampler's strided positions of
    the wrap-around padded index list; ``valid`` is False on padding copies."""
    items = rank_strided_indices(n_items, rank, world)
    per = len(items)
    valid = [rank + k * world < n_items for k in range(per)]
    return items, valid


def _collective_device(like):
    """gloo reduces host tensors, RCCL ("nccl") device tensors."""
    if dist.is_initialized() and dist.get_backend() == "nccl":
        return like.device
    return torch.device("cpu")


def allreduce_sum(t, world):
    if world == 1:
        return t
    d = _collective_device(t)
    x = t.to(d).clone()
    dist.all_reduce(x, op=dist.ReduceOp.SUM)
    return x.to(t.device)


def allgather_valid_rows(t, valid, world):
    """Rows of ``t`` ([n, ...], equal n on every rank) from all ranks, in
    rank order, keeping only the rows whose ``valid`` flag is set."""
    if world == 1:
        return t[valid.to(t.device)]
    d = _collective_device(t)
    parts = [torch.empty_like(t, device=d) for _ in range(world)]
    flags = [torch.empty_like(valid, device=d) for _ in range(world)]
    dist.all_gather(parts, t.to(d).contiguous())
    dist.all_gather(flags, valid.to(d).contiguous())
    return torch.cat([p[f.bool()] for p, f in zip(parts, flags)], 0)


def _batches(items, valid, batch_size):
    for i in range(0, len(items), batch_size):
        yield items[i:i + batch_size], valid[i:i + batch_size]


def _take(data, idx, device):
    ix = torch.as_tensor(idx, dtype=torch.long, device=data[0].device)
    return tuple(t.index_select(0, ix).to(device, non_blocking=True) for t in data)


class FusionFit:
    """``fit`` over tensor-backed datasets ``(dwi [N,14,S,S], dce [N,6,S,S],
    masks [N,1,32,32], labels [N])`` (host or device memory)."""

    def __init__(self, lm, train_data, val_data, batch_size=32, world=1, rank=0, use_graph=True, trainer=None):
        self.lm = lm
        self.train_data, self.val_data = train_data, val_data
        self.batch_size = batch_size
        self.world, self.rank = world, rank
        self.trainer = trainer if trainer is not None else FusionTrainer(lm, world=world, use_graph=use_graph)
        sc = self.trainer.lr_scheduler
        self.scheduler = sc["scheduler"] if isinstance(sc, dict) else sc
        self.monitor = sc.get("monitor", "val_loss") if isinstance(sc, dict) else "val_loss"
        self.history = []

    # ----------------------------------------------------------- training
    def train_epoch(self, epoch):
        lm = self.lm
        lm.current_epoch = epoch
        lm.on_train_epoch_start()
        lm.train()
        items, valid = shard(self.train_data[0].shape[0], self.rank, self.world)
        loss_sum = torch.zeros((), dtype=torch.float64, device=lm.device)
        steps = 0
        for idx, _ in _batches(items, valid, self.batch_size):
            loss = self.trainer.step(_take(self.train_data, idx, lm.device))
            loss_sum += loss.double()
            steps += 1
        tot = allreduce_sum(torch.stack([loss_sum, torch.tensor(float(steps), dtype=torch.float64,
                                                                device=lm.device)]), self.world)
        return (tot[0] / tot[1].clamp_min(1)).item()

    # --------------------------------------------------------- validation
    @torch.no_grad()
    def validate(self):
        lm = self.lm
        was = lm.training
        lm.eval()
        try:
            items, valid = shard(self.val_data[0].shape[0], self.rank, self.world)
            probs, labels, flags = [], [], []
            wsum = torch.zeros((), dtype=torch.float64, device=lm.device)
            nsum = torch.zeros((), dtype=torch.float64, device=lm.device)
            for idx, ok in _batches(items, valid, self.batch_size):
                nv = sum(ok)
                pad = len(idx) - nv
                flags.append(torch.tensor(ok, dtype=torch.uint8, device=lm.device))
                if nv == 0:
                    # a batch of padding copies only (e.g. n_val=65, world=2, batch 32: rank 1's last
                    # batch): nothing to score, but every rank must gather the same row count
                    probs.append(torch.zeros(pad, lm.class_num, dtype=torch.float32, device=lm.device))
                    labels.append(torch.zeros(pad, dtype=torch.long, device=lm.device))
                    continue
                # padding copies sit only at the end of the last batch: score the valid prefix
                batch = _take(self.val_data, idx[:nv], lm.device)
                loss, logits, _, _ = lm._shared_step(batch, phase="val", return_preds=True)
                wsum += loss.double() * nv
                nsum += nv
                p = torch.softmax(logits.float(), dim=1)
                if pad:
                    p = torch.cat([p, p.new_zeros(pad, p.shape[1])], 0)
                probs.append(p)
                labels.append(torch.cat([batch[-1].long(), batch[-1].new_zeros(pad).long()]))
            probs = torch.cat(probs, 0)
            labels = torch.cat(labels, 0)
            flags = torch.cat(flags, 0)
            tot = allreduce_sum(torch.stack([wsum, nsum]), self.world)
            val_loss = (tot[0] / tot[1]).item()
            all_p = allgather_valid_rows(probs, flags, self.world)
            all_y = allgather_valid_rows(labels, flags, self.world)
            auroc = metrics.multiclass_auroc(all_p, all_y, self.lm.class_num)
            acc = (all_p.argmax(1) == all_y).double().mean().item()
            return {"val_loss": val_loss, "val_roc_auc": auroc, "val_acc": acc, "n_val": int(all_y.numel()),
                    "probs": all_p.cpu(), "labels": all_y.cpu()}
        finally:
            lm.train(was)

    # ---------------------------------------------------------------- fit
    def fit(self, epochs, start_epoch=0):
        for epoch in range(start_epoch, start_epoch + epochs):
            train_loss = self.train_epoch(epoch)
            val = self.validate()
            if self.scheduler is not None:
                if isinstance(self.scheduler, torch.optim.lr_scheduler.ReduceLROnPlateau):
                    self.scheduler.step(val[self.monitor])
                else:
                    self.scheduler.step()
            rec = {"epoch": epoch, "train_loss": train_loss,
                   **{k: v for k, v in val.items() if k not in ("probs", "labels")},
                   "lr": [g["lr"] for g in self.trainer.opt.param_groups],
                   "captures": self.trainer.captures}
            if not math.isfinite(train_loss):
                raise RuntimeError(f"epoch {epoch}: non-finite training loss")
            self.history.append(rec)
        return self.history
