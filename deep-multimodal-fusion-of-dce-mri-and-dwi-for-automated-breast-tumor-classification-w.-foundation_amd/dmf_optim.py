"""Multi-tensor AdamW on the device -- drop-in for the ``torch.optim.AdamW``
that ``LightningFusionOptimizerFactory._get_base_optimizer`` builds
(selector_helpers.py:617-629, amsgrad=False).

One launch updates every parameter that has a gradient (parameters whose
grad is None are skipped, exactly like torch). Step counts and the per-group
hyper-parameters live in device memory, so a captured hipGraph replays the
update with the current values. ``pack_grads``/``grads_from`` let the
data-parallel driver all-reduce ONE flat gradient bucket and feed the
reduced bucket straight into the update (no unpack pass).
"""
from __future__ import annotations

import torch

import dmf_native as N
import dmf_ops as O

CHUNK = 8192


class FusedAdamW(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, amsgrad=False):
        if amsgrad:
            raise NotImplementedError("amsgrad is not used on the reference path")
        # torch.optim.AdamW's group keys too, so a saved state_dict loads into either optimizer
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=False, maximize=False,
                        foreach=None, capturable=False, differentiable=False, fused=None,
                        decoupled_weight_decay=True)
        super().__init__(params, defaults)
        self._table_key = None
        self._hyper = None
        self._hyper_host = None
        self._steps = None
        self._index = {}
        self.grad_source = None  # optional flat bucket (see pack_grads)
        self.grad_scale = 1.0
        self.tables_version = 0  # bumped whenever the device tables are rebuilt (captured graphs go stale)

    # -------------------------------------------------------------- tables
    def _live(self):
        out = []
        for gi, g in enumerate(self.param_groups):
            for p in g["params"]:
                if p.grad is not None or (self.grad_source is not None and p in self._bucket_offsets):
                    out.append((gi, p))
        return out

    def _hyper_values(self):
        vals = []
        for g in self.param_groups:
            b1, b2 = g["betas"]
            vals += [float(g["lr"]), float(g["weight_decay"]), float(b1), float(b2), float(g["eps"])]
        return vals

    def sync_hyper(self):
        vals = self._hyper_values()
        dev = self.param_groups[0]["params"][0].device
        if self._hyper is None or self._hyper.numel() != len(vals):
            self._hyper = torch.tensor(vals, dtype=torch.float32, device=dev)
            self._hyper_host = vals
        elif vals != self._hyper_host:
            self._hyper.copy_(torch.tensor(vals, dtype=torch.float32))
            self._hyper_host = vals

    def _build(self, live):
        dev = live[0][1].device
        # every param ever stepped keeps its slot (and step count) in _index;
        # moments loaded by load_state_dict are kept, and their 'step' seeds the slot
        seed = []
        for gi, p in live:
            if id(p) not in self._index:
                st = self.state[p]
                if "exp_avg" in st and "exp_avg_sq" in st:
                    for k in ("exp_avg", "exp_avg_sq"):
                        st[k] = st[k].to(device=p.device, dtype=torch.float32).contiguous()
                else:
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                slot = len(self._index)
                self._index[id(p)] = slot
                step0 = st.get("step", 0)
                step0 = int(step0.item()) if torch.is_tensor(step0) else int(step0)
                if step0:
                    seed.append((slot, step0))
        nslots = len(self._index)
        if self._steps is None or self._steps.numel() < nslots:
            old = self._steps
            self._steps = torch.zeros(max(nslots, 1), dtype=torch.int32, device=dev)
            if old is not None:
                self._steps[: old.numel()].copy_(old)
        if seed:
            idx = torch.tensor([a for a, _ in seed], dtype=torch.int64)
            val = torch.tensor([b for _, b in seed], dtype=torch.int32)
            self._steps[idx.to(dev)] = val.to(dev)
        rows, chunks = [], []
        slot_ids = []
        for t, (gi, p) in enumerate(live):
            if not p.is_contiguous():
                raise RuntimeError("FusedAdamW needs contiguous parameters")
            st = self.state[p]
            g = self._grad_ptr(p)
            rows.append([p.data_ptr(), g, st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr(), gi, p.numel()])
            slot_ids.append(self._index[id(p)])
            for b in range(0, p.numel(), CHUNK):
                chunks.append([t, b, min(p.numel(), b + CHUNK)])
        self._tensors = torch.tensor(rows, dtype=torch.int64, device=dev)
        self._chunks = torch.tensor(chunks, dtype=torch.int64, device=dev)
        self._nchunks = len(chunks)
        # per-live-tensor step counters: gather/scatter via a slot map kept on device
        self._slot = torch.tensor(slot_ids, dtype=torch.int64, device=dev)
        self._live_steps = self._steps[self._slot].clone()
        self.tables_version += 1

    def _grad_ptr(self, p):
        if self.grad_source is not None:
            off = self._bucket_offsets[p]
            return self.grad_source.data_ptr() + 4 * off
        if p.grad.dtype != torch.float32 or not p.grad.is_contiguous():
            raise RuntimeError("FusedAdamW needs contiguous fp32 gradients")
        return p.grad.data_ptr()

    def _key(self, live):
        return tuple((id(p), self._grad_ptr(p), p.data_ptr()) for _, p in live)

    # ---------------------------------------------------------------- step
    @torch.no_grad()
    def step(self, closure=None, scaler=None):
        """One AdamW update of every live tensor. With ``scaler`` (a
        DeviceGradScaler) the gradients are the scaled ones: a device-side
        inf / nan check runs first and, on overflow, the update and the step
        counters are skipped on the device; otherwise the update unscales by
        1/scale; then the scale is updated (GradScaler.step + update)."""
        loss = closure() if closure is not None else None
        live = self._live()
        if not live:
            return loss
        O.PREP.invalidate()  # the weights change: the step's batched conv re-layouts go stale
        capturing = torch.cuda.is_current_stream_capturing()
        if not capturing:
            self.sync_hyper()
            key = self._key(live)
            if key != self._table_key:
                if self._table_key is not None:
                    self._steps[self._slot] = self._live_steps
                self._build(live)
                self._table_key = key
        elif self._table_key is None:
            raise RuntimeError("run one eager optimizer step before capturing it in a graph")
        s = N.stream_ptr()
        if scaler is not None and scaler.enabled:
            N.call("dmf_amp_nonfinite", self._nchunks, self._chunks.data_ptr(), self._tensors.data_ptr(),
                   scaler.amp.data_ptr(), s)
            N.call("dmf_adamw_multi_amp", self._nchunks, self._chunks.data_ptr(), self._tensors.data_ptr(),
                   self._hyper.data_ptr(), self._live_steps.data_ptr(), self._live_steps.numel(),
                   float(self.grad_scale), scaler.amp.data_ptr(), s)
            scaler.update()
            return loss
        N.call("dmf_steps_inc", self._live_steps.data_ptr(), self._live_steps.numel(), s)
        N.call("dmf_adamw_multi", self._nchunks, self._chunks.data_ptr(), self._tensors.data_ptr(),
               self._hyper.data_ptr(), self._live_steps.data_ptr(), float(self.grad_scale), s)
        return loss

    @torch.no_grad()
    def zero_grad(self, set_to_none=False):
        if set_to_none:
            return super().zero_grad(set_to_none=True)
        pairs, chunks = [], []
        for g in self.param_groups:
            for p in g["params"]:
                if p.grad is not None:
                    t = len(pairs)
                    pairs.append([p.grad.data_ptr(), p.grad.data_ptr()])
                    for b in range(0, p.grad.numel(), CHUNK):
                        chunks.append([t, b, min(p.grad.numel(), b + CHUNK)])
        if not pairs:
            return
        key = tuple(x[0] for x in pairs)
        if getattr(self, "_zero_key", None) != key:
            dev = self.param_groups[0]["params"][0].device
            self._zero_pairs = torch.tensor(pairs, dtype=torch.int64, device=dev)
            self._zero_chunks = torch.tensor(chunks, dtype=torch.int64, device=dev)
            self._zero_key = key
        N.call("dmf_multi_copy", self._zero_chunks.shape[0], self._zero_chunks.data_ptr(), self._zero_pairs.data_ptr(),
               0.0, N.stream_ptr())

    def _flush_steps(self):
        """Device step counters -> self._steps (slot order)."""
        if self._table_key is not None:
            self._steps[self._slot] = self._live_steps

    def step_counts(self):
        """Per-parameter step counts (host copy; for tests)."""
        if self._table_key is None and self._steps is None:
            return {}
        self._flush_steps()
        return {i: int(v) for i, v in enumerate(self._steps.tolist())}

    # ---------------------------------------------------------- checkpoints
    def state_dict(self):
        """torch.optim.AdamW layout: per-parameter {'step' (float32 scalar
        tensor), 'exp_avg', 'exp_avg_sq'} -- the device step counters are
        written back into state[p]['step'] first, so the file loads into
        torch.optim.AdamW (what the reference's Lightning checkpoints hold)
        as well as into a FusedAdamW."""
        if self._steps is not None:
            self._flush_steps()
            host = self._steps.tolist()
            for g in self.param_groups:
                for p in g["params"]:
                    slot = self._index.get(id(p))
                    if slot is not None and p in self.state:
                        self.state[p]["step"] = torch.tensor(float(host[slot]), dtype=torch.float32)
        return super().state_dict()

    def load_state_dict(self, state_dict):
        """Replaces self.state (torch semantics) and drops every device table
        built over the old moment buffers: the next step rebuilds them over the
        loaded exp_avg / exp_avg_sq and seeds the step counters from 'step'."""
        super().load_state_dict(state_dict)
        self._table_key = None
        self._index = {}
        self._steps = None
        self._tensors = self._chunks = self._slot = self._live_steps = None
        self._hyper_host = None
        self.tables_version += 1

    # ----------------------------------------------------- flat grad bucket
    def make_bucket(self, params, segment_bytes=None, cuts=None):
        """Allocate ONE fp32 bucket laid out over ``params`` (the ones that
        receive gradients, in the order given); returns it. With
        ``segment_bytes`` the bucket is also cut into contiguous segments of
        about that size (``segments``: lists of param indices) that
        ``pack_segment`` fills one at a time -- the data-parallel driver
        all-reduces each as soon as its gradients are complete; ``cuts``
        (param counts) force segment boundaries. Use ``pack_grads`` (all of
        it) or ``pack_segment`` after backward."""
        self._bucket_params = list(params)
        self._bucket_offsets = {}
        off = 0
        for p in self._bucket_params:
            self._bucket_offsets[p] = off
            off += p.numel()
        dev = self._bucket_params[0].device
        self.bucket = torch.zeros(off, dtype=torch.float32, device=dev)
        self.segments, cur, size = [], [], 0
        limit = segment_bytes if segment_bytes else float("inf")
        cuts = set(cuts or ())
        for i, p in enumerate(self._bucket_params):
            cur.append(i)
            size += 4 * p.numel()
            if size >= limit or (i + 1) in cuts:
                self.segments.append(cur)
                cur, size = [], 0
        if cur:
            self.segments.append(cur)
        self._pack_key = None
        self._seg_tables = {}
        return self.bucket

    def segment_range(self, k):
        """(start, end) element range of segment k inside the bucket."""
        idx = self.segments[k]
        first, last = self._bucket_params[idx[0]], self._bucket_params[idx[-1]]
        return self._bucket_offsets[first], self._bucket_offsets[last] + last.numel()

    def _pack_tables(self, idx):
        pairs, chunks = [], []
        for t, i in enumerate(idx):
            p = self._bucket_params[i]
            if p.grad is None:
                raise RuntimeError("pack_grads: a bucket parameter has no gradient")
            pairs.append([p.grad.data_ptr(), self.bucket.data_ptr() + 4 * self._bucket_offsets[p]])
            for b in range(0, p.numel(), CHUNK):
                chunks.append([t, b, min(p.numel(), b + CHUNK)])
        return tuple(x[0] for x in pairs), pairs, chunks

    @torch.no_grad()
    def pack_grads(self):
        """bucket <- concat(p.grad) in one launch."""
        key, pairs, chunks = self._pack_tables(range(len(self._bucket_params)))
        if key != self._pack_key:
            dev = self.bucket.device
            self._pk_pairs = torch.tensor(pairs, dtype=torch.int64, device=dev)
            self._pk_chunks = torch.tensor(chunks, dtype=torch.int64, device=dev)
            self._pack_key = key
        N.call("dmf_multi_copy", self._pk_chunks.shape[0], self._pk_chunks.data_ptr(), self._pk_pairs.data_ptr(), 1.0,
               N.stream_ptr())

    @torch.no_grad()
    def pack_segment(self, k):
        """bucket[segment k] <- concat(p.grad of its params), one launch on
        the current stream (the device tables are built once per grad layout,
        outside any capture: call it eagerly once before capturing)."""
        key, pairs, chunks = self._pack_tables(self.segments[k])
        tab = self._seg_tables.get(k)
        if tab is None or tab[0] != key:
            dev = self.bucket.device
            tab = (key, torch.tensor(pairs, dtype=torch.int64, device=dev),
                   torch.tensor(chunks, dtype=torch.int64, device=dev))
            self._seg_tables[k] = tab
        N.call("dmf_multi_copy", tab[2].shape[0], tab[2].data_ptr(), tab[1].data_ptr(), 1.0, N.stream_ptr())

    def use_bucket_grads(self, enabled=True, scale=1.0):
        self.grad_source = self.bucket if enabled else None
        self.grad_scale = scale
        self._table_key = None if not enabled else self._table_key


class DeviceGradScaler:
    """torch.amp.GradScaler semantics for the captured step -- the reference
    trains with Lightning precision "16-mixed" (parameters_generate.py:211),
    i.e. autocast + GradScaler: the loss is scaled before backward, a step
    whose gradients overflow is skipped and the scale backs off (x0.5), and
    after ``growth_interval`` clean steps it grows (x2). Scale, growth tracker
    and the found-inf flag live on the device (no host sync, graph-replay
    safe): ``backward(loss)`` seeds autograd with the device scale,
    FusedAdamW.step(scaler=...) checks, unscales inside the update and
    updates the scale. The 16-bit MFMA type here is bf16 (fp32 range, so
    overflow skips are rare); the protocol is the reference's."""

    def __init__(self, device, init_scale=2.0 ** 16, growth_factor=2.0, backoff_factor=0.5, growth_interval=2000,
                 enabled=True):
        self.enabled = enabled
        self.growth_factor, self.backoff_factor, self.growth_interval = growth_factor, backoff_factor, growth_interval
        self.amp = torch.tensor([init_scale, 0.0], dtype=torch.float32, device=device)
        self.tracker = torch.zeros(1, dtype=torch.int32, device=device)

    def backward(self, loss):
        if not self.enabled:
            return loss.backward()
        if loss.dtype != torch.float32 or loss.dim() != 0:
            raise ValueError("DeviceGradScaler.backward: needs a scalar float32 loss")
        loss.backward(gradient=self.amp[0])

    def update(self):
        N.call("dmf_amp_update", self.amp.data_ptr(), self.tracker.data_ptr(), float(self.growth_factor),
               float(self.backoff_factor), int(self.growth_interval), N.stream_ptr())

    def get_scale(self):
        return float(self.amp[0].item())

    def state_dict(self):
        """torch.amp.GradScaler.state_dict layout."""
        return {"scale": self.get_scale(), "growth_factor": self.growth_factor, "backoff_factor": self.backoff_factor,
                "growth_interval": self.growth_interval, "_growth_tracker": int(self.tracker.item())}

    def load_state_dict(self, sd):
        with torch.no_grad():
            self.amp[0] = float(sd["scale"])
            self.amp[1] = 0.0
            self.tracker[0] = int(sd["_growth_tracker"])
        self.growth_factor = sd.get("growth_factor", self.growth_factor)
        self.backoff_factor = sd.get("backoff_factor", self.backoff_factor)
        self.growth_interval = sd.get("growth_interval", self.growth_interval)
