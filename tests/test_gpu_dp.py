"""The product's multi-rank training path on ONE GPU.

Two processes share cuda:0 and talk over gloo (RCCL refuses two ranks on one
device; the all-reduce is staged through the host, dmf_dp.allreduce_mean_).
Each runs ``FusionTrainer(world=2)`` -- captured hipGraphs, the packed fp32
gradient bucket, the eager all-reduce between the two graph halves and the
1/world grad_scale folded into AdamW -- on its rank-strided half of a B=8
batch, BN local; mode A (encoders frozen: the fusion bucket) and mode B
(everything trainable: the full bucket).

Reference: one process, the same seeded model, per-shard forward/backward
(local BN statistics per shard), the mean of the shard gradients, one step of
the product AdamW (eager, on p.grad; AdamW eps 1e-8 as the reference
configures it, see EPS) per training step. The two ranks must hold
bit-identical parameters, each rank's loss must be its shard's, and the
parameter change of every tensor must match the reference's to 1e-5 relative
L2, per tensor and over all parameters, in mode A and mode B: every reduction
of the step is fixed-order and (g0 + g1) * 0.5 is what both sides compute, so
the only freedom left is the exchange itself. A missing or doubled 1/world
scale moves every update by 2x and fails both bars.

Also single-process: a scheduler's learning-rate change reaches the captured
update, and a gradual unfreeze (new param group) re-captures the step so the
newly trainable parameters move (dmf_dp.py).

The RCCL path's overlapped exchange (post-accumulate-grad hooks launching
pack + ncclAllReduce per bucket segment on a comm stream, captured into the
step's hipGraph) runs here over a 1-rank RCCL communicator (dmf_rccl) -- the
only one a single GPU allows -- with small segments so the bucket is cut
many times:
the AdamW step reads ONLY the bucket, so a segment that was not packed and
reduced inside the replayed graph leaves stale gradients and the parameters
move away from the plain trainer's."""
import copy
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

STEPS = 2
B = 8
# The reference optimizer setting (AdamW eps 1e-8): AdamW's first steps are
# sign-like (g / (|g| + eps)), so this only holds because every gradient
# reduction of the step is fixed-order (test_gpu_determinism.py): the trainer's
# per-shard gradients are the eager reference's bit for bit, and what remains is
# the two AdamW implementations' rounding of the update.
EPS = 1e-8


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _build(dev, freeze=False, seed=0, eps=1e-8):
    import foundation_model as FM
    import model_module as MM
    import parameters as PR
    import train_fusion as TF
    from selector_helpers import get_classification_loss

    P = copy.deepcopy(PR.small_parameters(channels=(16, 32, 64), input_size=64, dropout=0.0))
    P["backbone_freeze_on_start"] = freeze
    P["dwi_model_parameters"]["optimizer_parameters"]["eps"] = eps
    P["dwi_model_parameters"]["compute_dtype"] = torch.float32
    torch.manual_seed(seed)
    bb = FM.build_medical_backbone(P, "cpu", "dwi", 14)
    dwi = MM.initialize_model(MM.ModelMaskHeadBackbone("dwi", P, bb), True)
    bb = FM.build_medical_backbone(P, "cpu", "dce", 6)
    dce = MM.initialize_model(MM.ModelMaskHeadBackbone("dce", P, bb), True)
    fm = MM.FusionModel(P)
    crit = get_classification_loss(P, torch.arange(64) % 4, "fusion", dev)
    lm = TF.LightningFusionModel(dwi.to(dev), dce.to(dev), fm.to(dev), P, crit)
    lm.train()
    return P, lm


def _batch(dev, seed):
    import make_golden as MG

    return tuple(t.to(dev) for t in MG.volume_batch(B, 64, seed))


def _worker(rank, world, port, outdir, mode):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dmf_dp import FusionTrainer, rank_strided_indices

        dev = torch.device("cuda", 0)
        _, lm = _build(dev, freeze=mode == "A", eps=EPS)
        tr = FusionTrainer(lm, world=world, use_graph=True)
        idx = torch.tensor(rank_strided_indices(B, rank, world), device=dev)
        losses = []
        for it in range(STEPS):
            local = tuple(t[idx] for t in _batch(dev, 40 + it))
            losses.append(float(tr.step(local).item()))
        torch.cuda.synchronize()
        params = {n: p.detach().cpu() for n, p in lm.named_parameters()}
        torch.save({"params": params, "losses": losses, "captures": tr.captures,
                    "bucket_numel": tr.opt.bucket.numel()}, os.path.join(outdir, f"rank{rank}.pt"))
    finally:
        dist.destroy_process_group()


def _reference(dev, world, mode):
    """Single process: mean of the per-shard gradients (local BN per shard), then
    torch.optim.AdamW with the same groups (selector_helpers.py:632-685)."""
    from dmf_dp import rank_strided_indices

    _, lm = _build(dev, freeze=mode == "A", eps=EPS)
    # the product's AdamW (dmf_optim.FusedAdamW, eager, on p.grad; its parity with torch.optim.AdamW is
    # test_gpu_parity.test_adamw_step_matches_torch): the trainer and this reference then differ only in
    # the data-parallel exchange under test
    cfg = lm.configure_optimizers()
    opt = cfg["optimizer"] if isinstance(cfg, dict) else cfg
    params = [p for g in opt.param_groups for p in g["params"]]
    losses = []
    for it in range(STEPS):
        full = _batch(dev, 40 + it)
        acc = [torch.zeros_like(p) for p in params]
        got = [False] * len(params)
        ls = []
        for r in range(world):
            idx = torch.tensor(rank_strided_indices(B, r, world), device=dev)
            for p in params:
                p.grad = None
            loss = lm.training_step(tuple(t[idx] for t in full))
            loss.backward()
            ls.append(float(loss.item()))
            for i, p in enumerate(params):
                if p.grad is not None:
                    acc[i] += p.grad.reshape(p.shape)
                    got[i] = True
        for i, p in enumerate(params):
            p.grad = acc[i] / world if got[i] else None
        opt.step()
        losses.append(ls)
    return {n: p.detach().cpu() for n, p in lm.named_parameters()}, losses


def _rel(a, b):
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.mark.timeout(900)
@pytest.mark.parametrize("mode", ["A", "B"])
def test_two_rank_fusion_trainer_matches_mean_gradient_step(tmp_path, mode):
    import parameters as PR  # noqa: F401  (import check before spawning)

    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_worker, args=(r, world, port, str(tmp_path), mode)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=600)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    r0 = torch.load(tmp_path / "rank0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "rank1.pt", weights_only=True)
    assert r0["captures"] == 1 and r0["bucket_numel"] > (1_000_000 if mode == "B" else 100_000)
    for n in r0["params"]:
        assert torch.equal(r0["params"][n], r1["params"][n]), n  # one bucket, one update: identical replicas
    _, lm0 = _build(torch.device("cpu"), freeze=mode == "A", eps=EPS)
    init = {n: p.detach().clone() for n, p in lm0.named_parameters()}
    want, ref_losses = _reference(torch.device("cuda", 0), world, mode)
    for it in range(STEPS):  # each rank's loss is its own shard's
        assert abs(r0["losses"][it] - ref_losses[it][0]) < 1e-4 * max(1, abs(ref_losses[it][0]))
        assert abs(r1["losses"][it] - ref_losses[it][1]) < 1e-4 * max(1, abs(ref_losses[it][1]))
    bad, d_got, d_want, pairs = {}, [], [], []
    for n, w in want.items():
        dw = w - init[n]
        if dw.abs().max().item() == 0:
            assert torch.equal(r0["params"][n].reshape(w.shape), w), n  # frozen / gradient-free stays put
            continue
        dg = r0["params"][n].reshape(w.shape) - init[n]
        d_got.append(dg.reshape(-1))
        d_want.append(dw.reshape(-1))
        pairs.append((n, dg, dw))
    gnorm = torch.cat(d_want).norm().item()
    for n, dg, dw in pairs:
        # tensors whose true gradient is zero (e.g. the GroupNorm biases ahead of
        # a conv -> train-mode BN, which removes any per-channel shift) move by
        # rounding noise only: judged by the global bar below, not per tensor
        if dw.norm().item() < 1e-4 * gnorm:
            continue
        e = _rel(dg, dw)
        if e > 1e-5:
            bad[n] = e
    assert not bad, sorted(bad.items(), key=lambda kv: -kv[1])[:10]
    tot = _rel(torch.cat(d_got), torch.cat(d_want))
    print(f"mode {mode}: relative L2 error of the parameter update over {len(d_got)} tensors: {tot:.2e}")
    assert tot < 1e-5, tot


def test_trainer_follows_lr_changes_and_unfreeze():
    from dmf_dp import FusionTrainer

    dev = torch.device("cuda", 0)
    P, lm = _build(dev, freeze=True)
    tr = FusionTrainer(lm, world=1, use_graph=True)
    b = _batch(dev, 7)
    before = {n: p.detach().clone() for n, p in lm.named_parameters()}
    bufs = {n: t.clone() for n, t in lm.named_buffers()}
    tr.capture(b)
    # capture's warm-up steps are undone: nothing trained, no BN statistics moved
    for n, p in lm.named_parameters():
        assert torch.equal(p.detach(), before[n]), n
    for n, t in lm.named_buffers():
        assert torch.equal(t, bufs[n]), n
    assert lm.global_step == 0
    tr.step(b)
    fus = [p for p in lm.fusion_model.parameters() if p.grad is not None]
    assert any(not torch.equal(p.detach(), before["fusion_model." + n])
               for n, p in lm.fusion_model.named_parameters() if p.grad is not None)
    # lr -> 0 (what ReduceLROnPlateau converges to): the replayed update must not move anything
    for g in tr.opt.param_groups:
        g["lr"] = 0.0
    snap = [p.detach().clone() for p in fus]
    tr.step(b)
    torch.cuda.synchronize()
    for p, s in zip(fus, snap):
        assert torch.equal(p.detach(), s)
    for g in tr.opt.param_groups:
        g["lr"] = 1e-4
    # gradual unfreeze at epoch 40 (selector_helpers.py:541-584): a new group -> re-capture
    enc_before = {n: p.detach().clone() for n, p in lm.dwi_model.named_parameters()}
    lm.current_epoch = P["unfreeze_timer"]
    lm.on_train_epoch_start()
    n_groups = len(tr.opt.param_groups)
    assert n_groups > 1
    caps = tr.captures
    tr.step(b)
    tr.step(b)
    torch.cuda.synchronize()
    assert tr.captures == caps + 1
    moved = [n for n, p in lm.dwi_model.named_parameters() if not torch.equal(p.detach(), enc_before[n])]
    assert moved, "no unfrozen encoder parameter was updated by the re-captured step"
    assert torch.isfinite(tr.loss).item()


def _overlap_worker(port, outdir, mode, prefork=False):
    import dmf_dp
    from dmf_dp import FusionTrainer

    dmf_dp.PREFORK = prefork
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    out = {}
    for tag, overlap in (("overlap", True), ("plain", False), ("plain2", False)):
        _, lm = _build(dev, freeze=mode == "A", eps=EPS)
        tr = FusionTrainer(lm, world=1, use_graph=True, overlap=overlap, bucket_mb=0.05)
        losses = []
        for it in range(3):
            losses.append(float(tr.step(_batch(dev, 60 + it)).item()))
        torch.cuda.synchronize()
        out[tag] = {"params": {n: p.detach().cpu() for n, p in lm.named_parameters()}, "losses": losses,
                    "captures": tr.captures, "segments": len(tr.opt.segments) if overlap else 0,
                    # segments whose all-reduce was launched from inside backward (not deferred to its end)
                    "early": (len(tr.opt.segments) - len(tr._deferred) - len(
                        [k for k in range(len(tr.opt.segments)) if tr._pending[k] > 0])) if overlap else 0}
    torch.save(out, os.path.join(outdir, "overlap.pt"))


@pytest.mark.timeout(600)
@pytest.mark.parametrize("mode,prefork", [("A", False), ("B", False), ("B", True)])
def test_overlapped_segment_allreduce_captured(tmp_path, mode, prefork):
    """prefork: the comm stream is forked from the step's stream at the start
    of backward, so the DCE encoder's segments (its own stream) join it by an
    event edge inside the capture instead of being deferred to the end."""
    ctx = mp.get_context("spawn")
    pr = ctx.Process(target=_overlap_worker, args=(_free_port(), str(tmp_path), mode, prefork))
    pr.start()
    pr.join(timeout=500)
    assert pr.exitcode == 0, pr.exitcode
    r = torch.load(tmp_path / "overlap.pt", weights_only=True)
    o, p = r["overlap"], r["plain"]
    assert o["captures"] == 1 and o["segments"] > 3, (o["captures"], o["segments"])
    # a 1-rank sum all-reduce is the identity and every reduction of the step is fixed-order: the
    # overlapped trainer's losses are the plain trainer's bit for bit
    assert o["losses"] == p["losses"] == r["plain2"]["losses"], (o["losses"], p["losses"], r["plain2"]["losses"])
    _, lm0 = _build(torch.device("cpu"), freeze=mode == "A", eps=EPS)
    init = {n: q.detach().clone() for n, q in lm0.named_parameters()}
    d_o, d_p = [], []
    for n, w in p["params"].items():
        dw = w - init[n]
        if dw.abs().max().item() == 0:
            assert torch.equal(o["params"][n], w), n
            continue
        d_o.append((o["params"][n] - init[n]).reshape(-1))
        d_p.append(dw.reshape(-1))
    tot = _rel(torch.cat(d_o), torch.cat(d_p))
    d_2 = [(r["plain2"]["params"][n] - init[n]).reshape(-1) for n, w in p["params"].items()
           if (w - init[n]).abs().max().item() != 0]
    noise = _rel(torch.cat(d_2), torch.cat(d_p))
    print(f"mode {mode} prefork {prefork}: overlapped vs plain update, relative L2 {tot:.2e} over {len(d_o)} "
          f"tensors (plain vs plain: {noise:.2e}); segments {o['segments']}, launched inside backward {o['early']}")
    # bit-identical parameters (AdamW eps 1e-8): the plain trainer reproduces itself exactly and the
    # overlapped, captured segment exchange changes nothing
    assert noise == 0.0 and tot == 0.0, (tot, noise)


def _aux_flip_worker(port, outdir):
    from dmf_dp import FusionTrainer

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    _, lm = _build(dev, freeze=True, eps=EPS)
    tr = FusionTrainer(lm, world=1, use_graph=True, overlap=True, bucket_mb=0.05)
    b = _batch(dev, 70)
    tr.step(b)
    before = (tr.captures, len(tr.opt.segments), tr.early_segments)
    lm.current_epoch = lm.aux_loss_limit  # aux_w = 0: the recon / mimic nodes drop out -> re-capture
    tr.step(b)
    tr.step(b)
    torch.cuda.synchronize()
    after = (tr.captures, len(tr.opt.segments), tr.early_segments)
    torch.save({"before": before, "after": after, "finite": bool(torch.isfinite(tr.loss).item())},
               os.path.join(outdir, "aux_flip.pt"))


@pytest.mark.timeout(600)
def test_overlap_survives_aux_gate_recapture(tmp_path):
    """a re-capture triggered by the aux-loss gate (epoch >= the
    aux limit) must re-learn the per-parameter ready-event counts. Doubled
    counts never reach zero, so every segment would be launched only at the
    end of backward and the overlap would be silently lost."""
    ctx = mp.get_context("spawn")
    pr = ctx.Process(target=_aux_flip_worker, args=(_free_port(), str(tmp_path)))
    pr.start()
    pr.join(timeout=500)
    assert pr.exitcode == 0, pr.exitcode
    r = torch.load(tmp_path / "aux_flip.pt", weights_only=True)
    (c0, s0, e0), (c1, s1, e1) = r["before"], r["after"]
    assert c0 == 1 and c1 == 2, (c0, c1)
    assert s0 > 3 and e0 > 0, (s0, e0)
    # segments still launch from inside backward after the re-capture (doubled counts: none would; the
    # recon / mimic heads' segments, without gradient once aux_w = 0, launch at its end)
    print(f"segments {s0} -> {s1}, launched inside backward {e0} -> {e1}")
    assert e1 > 0 and e1 >= s1 // 2, (s1, e1)
    assert r["finite"]


def test_short_first_batch_recaptures_on_full_batch():
    """a capture that lands on a short (ragged) batch must not make
    every later full-size batch run eagerly: the first larger batch re-captures
    the step; later short batches run eagerly beside the graph."""
    from dmf_dp import FusionTrainer

    dev = torch.device("cuda", 0)
    _, lm = _build(dev, freeze=True)
    tr = FusionTrainer(lm, world=1, use_graph=True)
    full = _batch(dev, 80)
    short = tuple(t[:3] for t in full)
    tr.step(short)
    assert tr.captures == 1
    with pytest.warns(RuntimeWarning, match="re-capturing"):
        tr.step(full)
    assert tr.captures == 2 and tr.static_batch[0].shape[0] == B
    tr.step(full)
    assert tr.captures == 2 and tr.eager_steps == 0
    tr.step(short)
    assert tr.eager_steps == 1 and tr.captures == 2
    torch.cuda.synchronize()
    assert torch.isfinite(tr.loss).item()


@pytest.mark.timeout(600)
def test_bench_gpus_2_spawns_two_ranks():
    """``bench.py --gpus N`` with no launcher starts N
    ranks itself (before touching the GPU) and rank 0 reports the whole job.
    Rehearsed on one GPU: two ranks share cuda:0 over gloo."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_PORT")}
    env.update(DMF_DIST_BACKEND="gloo", DMF_BENCH_SHARE_GPU="1")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
                        "--batch", "8", "--size", "128", "--no-extras", "--no-cpu-baseline", "--no-roofline"],
                       env=env, cwd=root, capture_output=True, text=True, timeout=540)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2" and d["config"]["global_batch"] == 16, d
    assert d["value"] > 0 and d["loss"] == d["loss"]


@pytest.mark.timeout(300)
def test_bench_gpus_n_without_share_needs_one_gpu_per_rank():
    """the exact branch the driver's ``--gpus 8`` takes (no
    launcher, no DMF_BENCH_SHARE_GPU): the parent spawns the ranks without
    touching HIP and each rank binds cuda:<local_rank>. On this one-GPU box
    rank 1's device does not exist: it must say so and exit non-zero, and the
    parent must stop rank 0 (blocked in the RCCL rendezvous) and fail."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_PORT", "DMF_BENCH_SHARE_GPU", "DMF_DIST_BACKEND")}
    if torch.cuda.device_count() >= 2:
        pytest.skip("more than one GPU visible: the two ranks would both find their device")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
                        "--batch", "4", "--size", "64", "--no-extras", "--no-cpu-baseline", "--no-roofline"],
                       env=env, cwd=root, capture_output=True, text=True, timeout=240)
    assert r.returncode != 0, r.stdout[-2000:]
    assert "cuda:1 is not visible" in r.stderr, r.stderr[-3000:]
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")], r.stdout[-2000:]
