#!/usr/bin/env python3
""""AUC vs ref" (VERDICT r01 item 6): a short config-3 mode-A
training run of the build next to the CPU oracle, same start and same data.

  * models: default_parameters() widths (128/256/512, ResNet-50 OS8 encoders,
    encoders frozen = mode A, the fusion model trains), dropout 0 so the two
    runs draw no random masks; the build runs in its fp32 parity mode
    (set_compute_dtype(float32)) through the product driver
    ``dmf_dp.FusionTrainer`` (captured hipGraph step, packed gradient bucket,
    fused AdamW), the oracle is ``oracle.losses.fusion_shared_step`` +
    ``torch.optim.AdamW`` over the same parameter groups;
  * data: a learnable synthetic set (``learnable_set``): a lesion disk whose
    DWI brightness and DCE enhancement curve (wash-in / plateau / wash-out
    shape) depend on the class, over noisy tissue; the mask target is the
    disk; fixed batch order;
  * the reference's validation metric: macro one-vs-rest AUROC of
    softmax(logits) over a held-out set (train.py:682-695,
    train_fusion.py:360), computed on the build side by ``metrics`` and on the
    oracle side by sklearn.

Reports the per-step training-loss trajectory of both runs, the val loss /
AUROC of both before and after training and their differences, and the
largest softmax-probability difference on the val set.

The run sweeps a 64-volume training set for 6 epochs (48 steps of B=8) at
lr 1e-3 on every group (the reference's 1e-4 needs far more steps than a
parity run affords to move a macro AUROC; both sides use the same value).

    python tools/auc_vs_ref.py [--steps 48] [--train 64] [--batch 8] [--size 128] [--val 48] [--lr 1e-3]
"""
import argparse
import copy
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "deep-multimodal-fusion-of-dce-mri-and-dwi-for-automated-breast-tumor-classification-w.-foundation_amd")
for p in (ROOT, PKG, os.path.join(ROOT, "tools")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

# DCE enhancement curve per class over the 6 phases (pre-contrast + 5 post):
# persistent rise, plateau, wash-out, weak -- the kinetic shapes a reader uses
CURVES = torch.tensor([[0.0, 0.10, 0.18, 0.25, 0.31, 0.36],
                       [0.0, 0.28, 0.33, 0.34, 0.34, 0.34],
                       [0.0, 0.40, 0.34, 0.27, 0.21, 0.16],
                       [0.0, 0.05, 0.07, 0.08, 0.09, 0.10]])


def learnable_set(n, S, seed, cd=14, cc=6):
    """n volumes, balanced classes in a seeded order -> (dwi, dce, masks, labels)."""
    g = torch.Generator().manual_seed(seed)
    labels = (torch.arange(n) % 4)[torch.randperm(n, generator=g)]
    yy, xx = torch.meshgrid(torch.arange(S, dtype=torch.float32), torch.arange(S, dtype=torch.float32),
                            indexing="ij")
    dwi = torch.empty(n, cd, S, S)
    dce = torch.empty(n, cc, S, S)
    masks = torch.zeros(n, 1, 32, 32)
    bvals = torch.linspace(0, 1, cd)
    for i in range(n):
        k = int(labels[i])
        cy, cx = (torch.rand(2, generator=g) * 0.5 + 0.25) * S
        r = S * (0.08 + 0.03 * k + 0.03 * torch.rand(1, generator=g).item())
        disk = ((((yy - cy) ** 2 + (xx - cx) ** 2) <= r * r).float())
        # DWI: restricted diffusion keeps lesion signal up at high b (class-dependent ADC)
        decay = torch.exp(-bvals * (0.5 + 0.6 * k))
        tissue = 0.35 * torch.exp(-bvals * 2.0)
        dwi[i] = (tissue[:, None, None] + disk * (0.45 * decay)[:, None, None]
                  + torch.randn(cd, S, S, generator=g) * 0.05).clamp(0, 1)
        dce[i] = (0.25 + disk * CURVES[k][:cc, None, None] * 1.6
                  + torch.randn(cc, S, S, generator=g) * 0.05).clamp(0, 1)
        masks[i, 0] = torch.nn.functional.interpolate(disk[None, None], size=(32, 32), mode="nearest")[0, 0]
    return dwi, dce, masks, labels


def _sklearn_auroc(probs, labels):
    from sklearn.metrics import roc_auc_score
    return float(roc_auc_score(labels, probs, multi_class="ovr", average="macro"))


def run(steps=48, batch=8, size=128, n_val=48, seed=0, n_train=64, lr=1e-3, device="cuda:0", log=print):
    import make_golden as MG
    import metrics as MT
    import model_module as MM
    import parameters as PR
    import train_fusion as TF
    from dmf_dp import FusionTrainer
    from oracle import losses as OL
    from selector_helpers import get_classification_loss

    dev = torch.device(device)
    P = copy.deepcopy(PR.default_parameters())
    P["dwi_model_parameters"]["dropout"] = 0.0
    P["dwi_model_parameters"]["input_size"] = size
    P["backbone_freeze_on_start"] = True
    dwi, dwi_r = MG.seeded_encoder(P, "dwi", 14, 71 + seed)
    dce, dce_r = MG.seeded_encoder(P, "dce", 6, 72 + seed)
    fm, fr = MG.seeded_fusion(P, 73 + seed)
    train = learnable_set(n_train, size, 1000 + seed)
    val = learnable_set(n_val, size, 2000 + seed)
    train_labels = train[3]

    # ---- build: fp32 parity mode through the product trainer
    for m in (dwi, dce, fm):
        MM.set_compute_dtype(m, torch.float32)
    crit = get_classification_loss(P, train_labels, "fusion", dev)
    lm = TF.LightningFusionModel(dwi.to(dev), dce.to(dev), fm.to(dev), P, crit)
    tr = FusionTrainer(lm, world=1, use_graph=True)
    for g in tr.opt.param_groups:
        g["lr"] = lr

    # ---- oracle: same state, torch.optim.AdamW over the build's groups
    ref = {"dwi_model.": dwi_r, "dce_model.": dce_r, "fusion_model.": fr}
    by_name = {pre + n: p for pre, m in ref.items() for n, p in m.named_parameters()}
    name_of = {id(p): n for n, p in lm.named_parameters()}
    groups = []
    for g in tr.opt.param_groups:
        ps = [by_name[name_of[id(p)]] for p in g["params"]]
        groups.append({"params": ps, "lr": g["lr"], "betas": g["betas"], "eps": g["eps"],
                       "weight_decay": g["weight_decay"]})
    trainable = {id(p) for g in groups for p in g["params"]}
    for p in by_name.values():
        p.requires_grad = id(p) in trainable
    opt_ref = torch.optim.AdamW(groups)
    cw = OL.class_weights_from_labels(train_labels)

    def evaluate():
        lm.eval()
        for m in ref.values():
            m.eval()
        pb, pr, lb, lr_ = [], [], [], []
        with torch.no_grad():
            for i in range(0, n_val, batch):
                bt = tuple(t[i:i + batch] for t in val)
                loss, logits, _, _ = lm._shared_step(tuple(t.to(dev) for t in bt), phase="val", return_preds=True)
                pb.append(torch.softmax(logits.float(), 1).cpu())
                lb.append(float(loss) * len(bt[3]))
                out = OL.fusion_shared_step(dwi_r, dce_r, fr, bt, P, cw, phase="val")
                pr.append(torch.softmax(out["logits"], 1))
                lr_.append(float(out["total"]) * len(bt[3]))
        lm.train()
        for m in ref.values():
            m.train()
        pb, pr = torch.cat(pb), torch.cat(pr)
        return {"auroc_build": MT.multiclass_auroc(pb, val[3], 4), "auroc_oracle": _sklearn_auroc(pr.numpy(),
                                                                                                  val[3].numpy()),
                "val_loss_build": sum(lb) / n_val, "val_loss_oracle": sum(lr_) / n_val,
                "max_prob_diff": (pb - pr).abs().max().item()}

    lm.train()
    for m in ref.values():
        m.train()
    t0 = time.time()
    before = evaluate()
    log(f"before: {json.dumps(before)}  ({time.time() - t0:.1f}s)")
    traj_b, traj_r, cls_r = [], [], []
    per_epoch = n_train // batch
    for it in range(steps):
        j = it % per_epoch
        bt = tuple(t[j * batch:(j + 1) * batch] for t in train)
        lb = float(tr.step(tuple(t.to(dev) for t in bt)).item())
        opt_ref.zero_grad(set_to_none=True)
        out = OL.fusion_shared_step(dwi_r, dce_r, fr, bt, P, cw, epoch=0)
        out["total"].backward()
        opt_ref.step()
        traj_b.append(lb)
        traj_r.append(float(out["total"]))
        cls_r.append(float(out["cls"]))
        if it % 4 == 0 or it == steps - 1:
            log(f"step {it:3d}: loss build {lb:.6f} oracle {traj_r[-1]:.6f}  ({time.time() - t0:.1f}s)")
    torch.cuda.synchronize()
    after = evaluate()
    log(f"after: {json.dumps(after)}  ({time.time() - t0:.1f}s)")
    tb, trf = np.array(traj_b), np.array(traj_r)
    return {
        "config": {"widths": list(P["dwi_model_parameters"]["channels"]), "size": size, "batch": batch,
                   "steps": steps, "n_train": n_train, "n_val": n_val, "lr": lr, "mode": "A (encoders frozen)", "compute": "fp32 parity mode",
                   "seed": seed},
        "loss_build": traj_b, "loss_oracle": traj_r, "loss_oracle_cls": cls_r,
        "max_abs_loss_diff": float(np.abs(tb - trf).max()),
        "max_rel_loss_diff": float((np.abs(tb - trf) / np.abs(trf)).max()),
        "before": before, "after": after,
        "auroc_diff": abs(after["auroc_build"] - after["auroc_oracle"]),
        "val_loss_rel_diff": abs(after["val_loss_build"] - after["val_loss_oracle"]) / abs(after["val_loss_oracle"]),
        "seconds": round(time.time() - t0, 1),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=48)
    ap.add_argument("--train", type=int, default=64)
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--size", type=int, default=128)
    ap.add_argument("--val", type=int, default=48)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "auc_vs_ref.json"))
    a = ap.parse_args()
    torch.set_num_threads(int(os.environ.get("OMP_NUM_THREADS", "16")))
    rep = run(a.steps, a.batch, a.size, a.val, a.seed, a.train, a.lr)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(rep, f, indent=1)
    print(json.dumps({k: v for k, v in rep.items() if not k.startswith("loss_")}))


if __name__ == "__main__":
    main()
