"""The product's epoch driver (dmf_fit.FusionFit, VERDICT r02 "Next" 6) on two
ranks sharing one GPU over gloo, against the same driver in one process.

* Validation is exact under sharding: each rank scores its strided shard
  (eval-mode BN, no dropout), the probabilities and labels are all-gathered
  (padding rows dropped) and the macro OvR AUROC over the whole epoch equals
  the single-process AUROC over the same validation set; the sample-weighted
  val_loss (Lightning's on_epoch mean, train.py:1058-1066) is all-reduced
  and equals the single-process value (reference: train.py:682-695,
  train_fusion.py:342-405).
* A two-epoch fit with unfreeze every epoch (selector_helpers.py:541-584):
  the step is re-captured at the unfreeze, ReduceLROnPlateau receives the
  all-reduced val_loss (selector_helpers.py:148-156), and both ranks end
  with bit-identical parameters, learning rates and epoch metrics.
"""
import copy
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

N_TRAIN, N_VAL, S, B = 14, 11, 64, 4


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _build(dev):
    import foundation_model as FM
    import model_module as MM
    import parameters as PR
    import train_fusion as TF
    from selector_helpers import get_classification_loss

    P = copy.deepcopy(PR.small_parameters(channels=(16, 32, 64), input_size=S, dropout=0.0))
    P["dwi_model_parameters"]["compute_dtype"] = torch.float32
    P["unfreeze_timer"] = 1
    P["dwi_model_parameters"]["scheduler"]["patience"] = 0
    torch.manual_seed(0)
    bb = FM.build_medical_backbone(P, "cpu", "dwi", 14)
    dwi = MM.initialize_model(MM.ModelMaskHeadBackbone("dwi", P, bb), True)
    bb = FM.build_medical_backbone(P, "cpu", "dce", 6)
    dce = MM.initialize_model(MM.ModelMaskHeadBackbone("dce", P, bb), True)
    fm = MM.FusionModel(P)
    crit = get_classification_loss(P, torch.arange(64) % 4, "fusion", dev)
    lm = TF.LightningFusionModel(dwi.to(dev), dce.to(dev), fm.to(dev), P, crit)
    lm.train()
    return lm


def _data(n, seed):
    import make_golden as MG

    d = MG.volume_batch(n, S, seed)
    return tuple(t for t in d)


def _run(world, rank, outdir):
    from dmf_fit import FusionFit

    dev = torch.device("cuda", 0)
    lm = _build(dev)
    fit = FusionFit(lm, _data(N_TRAIN, 90), _data(N_VAL, 91), batch_size=B, world=world, rank=rank)
    v0 = fit.validate()
    hist = fit.fit(2)
    torch.cuda.synchronize()
    out = {"val0": {k: v for k, v in v0.items()}, "hist": hist,
           "params": {n: p.detach().cpu() for n, p in lm.named_parameters()}}
    torch.save(out, os.path.join(outdir, f"fit_w{world}_r{rank}.pt"))


def _worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        _run(world, rank, outdir)
    finally:
        dist.destroy_process_group()


def _single(outdir):
    _run(1, 0, outdir)


@pytest.mark.timeout(900)
def test_fit_two_ranks_validation_exact_and_epochs_consistent(tmp_path):
    import parameters as PR  # noqa: F401  (import check before spawning)

    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, str(tmp_path))) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=700)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    one = ctx.Process(target=_single, args=(str(tmp_path),))
    one.start()
    one.join(timeout=500)
    assert one.exitcode == 0, one.exitcode
    r0 = torch.load(tmp_path / "fit_w2_r0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "fit_w2_r1.pt", weights_only=True)
    s1 = torch.load(tmp_path / "fit_w1_r0.pt", weights_only=True)
    # validation before any training: sharded == single process, over all N_VAL volumes
    for r in (r0, r1):
        assert r["val0"]["n_val"] == N_VAL
        assert abs(r["val0"]["val_roc_auc"] - s1["val0"]["val_roc_auc"]) < 1e-9, (r["val0"], s1["val0"])
        assert abs(r["val0"]["val_loss"] - s1["val0"]["val_loss"]) <= 1e-6 * abs(s1["val0"]["val_loss"])
        assert torch.allclose(r["val0"]["probs"].sort(0).values, s1["val0"]["probs"].sort(0).values, atol=1e-6)
    print("val before training: AUROC", r0["val0"]["val_roc_auc"], "loss", r0["val0"]["val_loss"])
    # two epochs: re-capture at the unfreeze, identical replicas and metrics on both ranks
    h0, h1 = r0["hist"], r1["hist"]
    assert [h["epoch"] for h in h0] == [0, 1]
    assert h0[-1]["captures"] == 2, [h["captures"] for h in h0]
    for a, b in zip(h0, h1):
        for k in ("train_loss", "val_loss", "val_roc_auc", "val_acc", "lr"):
            assert a[k] == b[k], (k, a[k], b[k])
    assert len(h0[-1]["lr"]) > 1  # a backbone group was added at the epoch-1 unfreeze
    for n in r0["params"]:
        assert torch.equal(r0["params"][n], r1["params"][n]), n
    print("fit history:", [{k: h[k] for k in ("epoch", "train_loss", "val_loss", "val_roc_auc", "lr")} for h in h0])
