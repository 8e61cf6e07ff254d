"""Data-parallel fusion training driver (one process per GPU, RCCL over xGMI).

Replaces the Lightning Trainer that ``run_training.run_fusion_model``
(run_training.py:181-333) builds, for the hot path only:
  * rank-strided sampling of volumes (each rank its own local batch; BN stays
    LOCAL, as the reference uses plain BatchNorm2d -- SURVEY.md 8(e));
  * the gradients of every trainable parameter go to ONE flat fp32 bucket
    that the AdamW kernel reads directly with scale 1/world (no unpack pass);
  * with RCCL (backend "nccl") the exchange OVERLAPS the backward: the bucket
    is laid out in gradient-ready order and cut into ~bucket_mb (32 MB)
    segments; a post-accumulate-grad hook launches pack + ``all_reduce`` of a
    segment on a communication stream the moment its last gradient lands,
    while autograd keeps computing the earlier layers' gradients (fusion
    model first, then the encoders' heads, layer4 ... stem). The collectives
    run on a bare RCCL communicator (dmf_rccl) and are captured into the
    step's hipGraph with everything else (RCCL supports stream capture;
    probed in tools/capture_fork_probe.py);
  * with gloo (the CPU / shared-GPU rehearsal) the bucket is packed after
    backward and all-reduced once, eagerly, between the two captured graphs;
  * the step (forward + backward [+ exchange] + AdamW) is captured into
    hipGraphs after warm-up, so the Python launch overhead is paid once;
  * epoch-end AUROC over the all-gathered probabilities (metrics.py).
"""
from __future__ import annotations

import os
import warnings

import torch
import torch.distributed as dist


def dist_env():
    """(rank, local_rank, world) from the torchrun environment (1-process defaults)."""
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("LOCAL_RANK", 0)),
            int(os.environ.get("WORLD_SIZE", 1)))


# PREFORK (knob "dp_prefork", default): the comm stream is forked from the step's
# stream when backward begins, so a segment produced on the DCE encoder's stream
# only adds an event edge into an already-forked branch and overlaps the rest of
# backward inside the captured graph too
# (tests/test_gpu_dp.py::test_overlapped_segment_allreduce_captured[B-True]).
# Without it such segments are deferred to the end of backward during capture: a
# comm stream forked from the concurrent DCE encoder stream (a fork of a fork)
# crashes torch 2.10 + HIP 7 at capture end when aten kernels run on the nested
# stream (tools/capture_fork_probe.py)
PREFORK = True


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
        if bucket.is_cuda and dist.get_backend(group) == "gloo":
            # gloo (CPU rehearsal of the multi-rank path, e.g. two ranks sharing
            # one GPU): stage through the host
            host = bucket.cpu()
            dist.all_reduce(host, op=dist.ReduceOp.SUM, group=group)
            bucket.copy_(host)
        else:
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
    captured step. ``step(batch)`` runs one training step.

    The captured graphs hold device pointers of the optimizer tables, the
    hyper-parameter table and the gradient bucket. ``step`` therefore
    (i) writes the current learning rates / weight decays into the existing
    hyper table before every replay (a scheduler's changes reach the device),
    and (ii) drops the graphs and the bucket whenever the trainable set, the
    param-group layout or the optimizer's tables change (gradual unfreeze,
    selector_helpers.py:541-613; load_state_dict), re-capturing on that step's
    batch -- capture restores the training state its warm-up steps touched, so
    it never advances training."""

    def __init__(self, lm, world=1, use_graph=True, overlap=None, bucket_mb=None):
        self.lm = lm
        self.world = world
        self.use_graph = use_graph
        if overlap is None:
            overlap = world > 1 and dist.is_initialized() and dist.get_backend() == "nccl"
        # overlap=True with world=1 runs the same hooks / segments / captured
        # collectives over a 1-rank communicator (the single-GPU test of the path)
        self.overlap = bool(overlap)
        mb = bucket_mb if bucket_mb is not None else 32.0
        self.segment_bytes = int(mb * (1 << 20))
        self._hooks = []
        self._ready_order = []
        self._fires = {}
        self._armed = False
        self._comm = None
        self._rccl = None
        # Lightning precision "16-mixed" (the reference's default,
        # parameters_generate.py:211): dynamic loss scaling on the device
        self.scaler = None
        if lm.parameters_dict.get("precision") in ("16-mixed", "16"):
            from dmf_optim import DeviceGradScaler
            self.scaler = DeviceGradScaler(lm.device)
        cfg = lm.configure_optimizers()
        self.opt = cfg["optimizer"] if isinstance(cfg, dict) else cfg
        # {"scheduler", "monitor", "interval"} of the factory (selector_helpers.py:148-156), stepped by the
        # epoch driver (dmf_fit.FusionFit) with the all-reduced val_loss
        self.lr_scheduler = cfg.get("lr_scheduler") if isinstance(cfg, dict) else None
        self.lm.optimizer = self.opt
        self.graphs = None
        self.static_batch = None
        self._bucket_ready = False
        self._bucket_sig = None
        self._graph_sig = None
        self.loss = None
        self.captures = 0
        self.eager_steps = 0  # steps that ran eagerly beside a captured graph (shape mismatch)
        self.early_segments = 0

    # ------------------------------------------------------------ signature
    def _trainable(self):
        return [p for g in self.opt.param_groups for p in g["params"] if p.requires_grad]

    def _signature(self):
        groups = tuple(len(g["params"]) for g in self.opt.param_groups)
        step_sig = self.lm.step_signature() if hasattr(self.lm, "step_signature") else ()
        return groups, tuple(id(p) for p in self._trainable()), self.opt.tables_version, step_sig

    # ------------------------------------------------- overlapped exchange
    def _install_hooks(self):
        import dmf_ops as O

        for h in self._hooks:
            h.remove()
        self._hooks = [p.register_post_accumulate_grad_hook(self._on_grad) for p in self._trainable()]
        # conv weights and BN gamma / beta get their gradients through grad_sink (no AccumulateGrad,
        # so no post-accumulate hook): the sink path reports them once their kernels are enqueued.
        # Registered weakly: a dropped trainer (and its model / optimizer) is not kept alive by the
        # module-global list
        O.add_sink_hook(self._on_grad)
        self._fires = {}

    def _on_grad(self, p):
        if not self._armed:
            return
        if not self._bucket_ready:
            # first step: learn the gradient-ready order, the stream each gradient is produced on
            # (DWI / fusion: the step's stream; DCE: its concurrent encoder stream) and how many
            # ready events each parameter raises per step
            if id(p) not in self._fires:
                self._ready_order.append((p, torch.cuda.current_stream().cuda_stream))
            self._fires[id(p)] = self._fires.get(id(p), 0) + 1
            return
        k = self._seg_of.get(p)
        if k is None:
            return
        self._pending[k] -= 1
        if self._pending[k] == 0:
            self._launch_segment(k)

    def _launch_segment(self, k):
        """pack + all_reduce segment k on the comm stream, forked from the
        stream its last gradient was produced on. A gradient made on a side
        stream (the concurrent DCE encoder) is deferred to the end of
        backward while a graph is being captured: a fork from a forked stream
        breaks capture end on this stack."""
        cur = torch.cuda.current_stream()
        if torch.cuda.is_current_stream_capturing() and cur != self._origin and not PREFORK:
            self._deferred.append(k)
            return
        self._launched.add(k)
        self._comm.wait_stream(cur)
        with torch.cuda.stream(self._comm):
            self.opt.pack_segment(k)
            a, b = self.opt.segment_range(k)
            self._rccl.all_reduce_sum_(self.opt.bucket[a:b])

    def _begin_backward(self):
        self._origin = torch.cuda.current_stream()
        if self._comm is None:
            from dmf_rccl import RcclComm
            self._comm = torch.cuda.Stream(self._origin.device)
            rank = dist.get_rank() if dist.is_initialized() else 0
            self._rccl = RcclComm(rank, self.world, self._origin.device)
        if self._bucket_ready:
            # ready events per segment (a parameter may raise more than one: learned in the first step)
            self._pending = [sum(self._fires.get(id(self.opt._bucket_params[i]), 1) for i in seg)
                             for seg in self.opt.segments]
        self._launched, self._deferred = set(), []
        if PREFORK:
            self._comm.wait_stream(self._origin)
        self._armed = True

    def _end_backward(self):
        self._armed = False
        # segments whose exchange was launched from inside backward (overlapped); of a captured step,
        # this is the count its graph holds
        self.early_segments = len(self._launched)
        if not self._bucket_ready or self._bucket_sig != self._signature()[:2]:
            self._setup_bucket()
        # segments whose params got no gradient this step, and deferred ones
        for k in range(len(self.opt.segments)):
            if k not in self._launched:
                self._launch_segment(k)
        self._origin.wait_stream(self._comm)

    # ---------------------------------------------------------- eager step
    def _fwd_bwd(self, batch):
        self.opt.zero_grad(set_to_none=False)
        loss = self.lm.training_step(batch)
        bwd = self.scaler.backward if self.scaler is not None else (lambda t: t.backward())
        import dmf_ops as O

        # both encoders differentiate (mode B) AND the forward forked them onto two streams
        # (train_fusion._encode): only then do their backwards run concurrently and the dgrad
        # launches take half-chip tiles; a serial forward keeps chip-filling launches
        two = (self.lm.__dict__.get("_encoders_forked", False)
               and all(any(p.requires_grad for p in m.parameters())
                       for m in (self.lm.dwi_model, self.lm.dce_model)))
        if two:
            O.concurrent_tiles(True, bwd=True)
        try:
            if self.overlap:
                self._begin_backward()
                bwd(loss)
                self._end_backward()
            else:
                bwd(loss)
        finally:
            if two:
                O.concurrent_tiles(False, bwd=True)

        if O.GRAD_STASH:
            # a full backward consumes every shortcut-gradient hand-off (dmf_ops.conv_bn_act)
            n = len(O.GRAD_STASH)
            O.GRAD_STASH.clear()
            raise RuntimeError(f"{n} shortcut gradient hand-off(s) left undelivered by the training backward")
        return loss

    def _exchange_and_update(self):
        if self.world > 1 and not self.overlap:
            self.opt.pack_grads()
            allreduce_mean_(self.opt.bucket, self.world)
        self.opt.step(scaler=self.scaler)

    def _setup_bucket(self):
        params = [p for p in self._trainable() if p.grad is not None]
        if self.overlap and self._ready_order:
            # gradient-ready order (what backward produced first is reduced
            # first), one run per producing stream: a segment never mixes
            # gradients of two concurrent streams, so it is launched from the
            # stream that made all of its gradients; anything not seen last
            runs = {}
            for p, sid in self._ready_order:
                if p.grad is not None and p.requires_grad:
                    runs.setdefault(sid, []).append(p)
            seen = {id(p) for p, _ in self._ready_order}
            params = [p for run in runs.values() for p in run] + [p for p in params if id(p) not in seen]
            cuts = []
            n = 0
            for run in runs.values():
                n += len(run)
                cuts.append(n)
        if self.world > 1 or self.overlap:
            self.opt.use_bucket_grads(False)
            if params:
                self.opt.make_bucket(params, self.segment_bytes if self.overlap else None,
                                     cuts if self.overlap and self._ready_order else None)
                self.opt.use_bucket_grads(True, 1.0 / self.world)
                if self.overlap:
                    self._seg_of = {p: k for k, seg in enumerate(self.opt.segments)
                                    for i in seg for p in (self.opt._bucket_params[i],)}
        self._bucket_ready = True
        self._bucket_sig = self._signature()[:2]

    def eager_step(self, batch):
        if self.overlap and (not self._hooks or not self._bucket_ready or self._bucket_sig != self._signature()[:2]):
            # a (re-)learning step: fresh hooks and per-parameter ready-event counts. Every re-capture
            # (aux-loss gate flip, optimizer tables) clears _bucket_ready and lands here, so its warm-up
            # never adds a second round of counts on top of the old ones (doubled
            # _pending totals never reach 0 and every segment would wait for _end_backward)
            self._install_hooks()
            self._bucket_ready = False
            self._ready_order = []
        loss = self._fwd_bwd(batch)
        if not self._bucket_ready or self._bucket_sig != self._signature()[:2]:
            self._setup_bucket()
        self._exchange_and_update()
        self.lm.global_step += 1
        self.loss = loss.detach()
        return loss

    # ------------------------------------------------------------- state
    def _snapshot(self):
        """Device copies of everything a training step mutates: trainable
        parameters, every buffer (BN running stats, num_batches_tracked), the
        optimizer moments and step counters, the dropout Philox states."""
        import dmf_ops as O

        o = self.opt
        return {"params": [(p, p.detach().clone()) for p in self._trainable()],
                "buffers": [(b, b.clone()) for _, b in self.lm.named_buffers()],
                "opt": {id(t): (t, t.clone()) for st in o.state.values() for t in st.values()
                        if torch.is_tensor(t) and t.is_cuda},
                "steps": self._steps_by_param(),
                "rng": [(t, t.clone()) for t in O.RNG.states.values()]
                + ([(self.scaler.amp, self.scaler.amp.clone()), (self.scaler.tracker, self.scaler.tracker.clone())]
                   if self.scaler is not None else []),
                "global_step": self.lm.global_step}

    def _steps_by_param(self):
        """{id(param): AdamW step count} as the optimizer would continue from:
        the device counters where a slot exists, else the state's 'step'
        (e.g. just after load_state_dict)."""
        o = self.opt
        dev_steps = None
        if o._steps is not None:
            o._flush_steps()
            dev_steps = o._steps.tolist()
        out = {}
        for g in o.param_groups:
            for p in g["params"]:
                slot = o._index.get(id(p))
                if slot is not None and dev_steps is not None:
                    out[id(p)] = int(dev_steps[slot])
                elif p in o.state and "step" in o.state[p]:
                    st = o.state[p]["step"]
                    out[id(p)] = int(st.item() if torch.is_tensor(st) else st)
        return out

    def _restore(self, snap):
        """Undo what the steps since ``snap`` changed, in place (the captured
        graphs keep pointing at the same storage). Moments created after the
        snapshot go back to zero, step counters to their snapshot values."""
        o = self.opt
        with torch.no_grad():
            for key in ("params", "buffers", "rng"):
                for t, v in snap[key]:
                    t.copy_(v)
            saved = snap["opt"]
            for st in o.state.values():
                for t in st.values():
                    if torch.is_tensor(t) and t.is_cuda:
                        if id(t) in saved:
                            t.copy_(saved[id(t)][1])
                        else:
                            t.zero_()
            if o._steps is not None:
                # every slot back to its parameter's count at the snapshot: a slot seeded from a
                # loaded checkpoint's 'step' (load_state_dict leaves _steps unset until the warm-up
                # steps build it) returns to that value, a slot that did not exist to 0
                want = torch.zeros(o._steps.numel(), dtype=torch.int32)
                for pid, slot in o._index.items():
                    want[slot] = snap["steps"].get(pid, 0)
                want = want.to(o._steps.device)
                o._steps.copy_(want)
                if o._table_key is not None and o._live_steps is not None:
                    o._live_steps.copy_(want[o._slot])
        self.lm.global_step = snap["global_step"]

    # ----------------------------------------------------------- graphs
    def capture(self, batch):
        """Capture fwd+bwd(+pack) and the update as hipGraphs. With overlap
        the segment all-reduces are inside the first graph; otherwise (gloo)
        the one all-reduce stays eager between the two. The two eager
        warm-up steps (allocator pools, weight caches, optimizer and pack
        tables, the gradient-ready order) are undone afterwards, so capture
        leaves the parameters, buffers, optimizer state, RNG and global_step
        as it found them."""
        self.static_batch = tuple(t.clone() for t in batch)
        torch.cuda.synchronize()
        snap = self._snapshot()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):  # warm the allocator / tables on the side stream
                self.eager_step(self.static_batch)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        g1 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g1):
            # detached: keeping the capture pass's autograd graph alive would pin its saved
            # activations (and trips torch's AccumulateGrad stream check on later steps)
            self._graph_loss = self._fwd_bwd(self.static_batch).detach()
            if self.world > 1 and not self.overlap:
                self.opt.pack_grads()
        g2 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g2):
            self.opt.step(scaler=self.scaler)
        self.graphs = (g1, g2)
        self.loss = self._graph_loss
        self._restore(snap)
        torch.cuda.synchronize()
        self._graph_sig = self._signature()
        self.captures += 1

    def _rows(self, batch):
        return batch[0].shape[0] if batch is not None else 0

    def step(self, batch=None):
        if self.graphs is not None and self._graph_sig != self._signature():
            # unfreeze / new param group / reloaded optimizer: the captured
            # pointers are stale -- rebuild the bucket and capture again, on a
            # full-size batch: a ragged one (an epoch's last) would make every later
            # full batch miss the captured shapes; the previous static batch is
            # full-size, and capture leaves the training state untouched
            self.graphs = None
            self._bucket_ready = False
            if self.use_graph:
                full = batch if self._rows(batch) >= self._rows(self.static_batch) else self.static_batch
                self.capture(full)
        if self.graphs is None:
            if self.use_graph and self.captures == 0 and batch is not None:
                self.capture(batch)
            else:
                return self.eager_step(batch)
        if batch is not None and any(a.shape != b.shape for a, b in zip(batch, self.static_batch)):
            if self.use_graph and self._rows(batch) > self._rows(self.static_batch):
                # the first capture landed on a short batch: capture again on this larger one, so the
                # full-size batches replay instead of falling back to eager for the rest of training
                warnings.warn(f"re-capturing the training step: batch of {self._rows(batch)} volumes after a capture "
                              f"on {self._rows(self.static_batch)}", RuntimeWarning)
                self.graphs = None
                self._bucket_ready = False
                self.capture(batch)
            else:
                # a ragged batch (an epoch's last one): the captured shapes do not apply -- run it eagerly
                self.eager_steps += 1
                return self.eager_step(batch)
        if batch is not None and batch[0].data_ptr() != self.static_batch[0].data_ptr():
            for dst, src in zip(self.static_batch, batch):
                dst.copy_(src, non_blocking=True)
        self.opt.sync_hyper()  # scheduler lr / wd changes -> the captured hyper table (same storage)
        if hasattr(self.lm, "sync_step_scalars"):
            self.lm.sync_step_scalars()  # the epoch's aux-loss weight -> the scalar the captured loss reads
        g1, g2 = self.graphs
        g1.replay()
        if self.world > 1 and not self.overlap:
            allreduce_mean_(self.opt.bucket, self.world)
        g2.replay()
        self.lm.global_step += 1
        self.loss = self._graph_loss  # (an eager ragged step in between rebinds self.loss)
        return self.loss
