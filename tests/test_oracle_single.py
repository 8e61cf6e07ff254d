"""CPU: the oracle's single-modality step (oracle/losses.py single_shared_step,
reference train.py:294-466) assembles its terms as the reference does --
recon/mimic weighted twice by lambda * aux_w in training (train.py:400-403
after :458-460), recon SUMMED over recon_feats, feat-norm on the encoder's
raw_feats, nothing but the classification term in validation. Parity of the
individual criteria is pinned by the golden vectors (test_oracle_golden.py)."""
import copy

import torch

import foundation_model as FM
import model_module as MM
import parameters as PR
from oracle import losses as OL
from oracle import model as OM


def _oracle_encoder(seed=5):
    P = PR.small_parameters(dropout=0.0)
    torch.manual_seed(seed)
    P = copy.deepcopy(P)
    bb = FM.build_medical_backbone(P, "cpu", "dwi", 14)
    enc = MM.initialize_model(MM.ModelMaskHeadBackbone("dwi", P, bb), True)
    ref = OM.ModelMaskHeadBackbone("dwi", P, OM.ResNet50OS8(14))
    ref.load_state_dict(enc.state_dict())
    return ref, P


def test_single_step_assembly_quirks():
    ref, P = _oracle_encoder()
    ref.eval()  # deterministic BN so the two evaluations see the same forward
    g = torch.Generator().manual_seed(1)
    x = (0.5 + torch.randn(4, 14, 64, 64, generator=g) / 6).clamp(0, 1)
    m = (torch.rand(4, 1, 32, 32, generator=g) > 0.5).float()
    y = torch.tensor([0, 1, 2, 3])
    cw = OL.class_weights_from_labels(torch.arange(64) % 4)
    mp = P["dwi_model_parameters"]
    epoch = 20
    aux_w = 1 - epoch / P["aux_loss_weight_epoch_limit"]
    with torch.no_grad():
        r = OL.single_shared_step(ref, (x, m, y), P, cw, "dwi", epoch=epoch)
        v = OL.single_shared_step(ref, (x, m, y), P, cw, "dwi", epoch=epoch, phase="val")
        logits, aux, mask = ref(x)
    lr, lm = mp["lambda_recon"], mp["lambda_mimic"]
    raw_recon = sum(OL.recon_image_loss(torch.nn.functional.interpolate(rr, size=(64, 64), mode="bilinear",
                                                                        align_corners=False),
                                        x.mean(1, keepdim=True)) for rr in aux["recon_feats"])
    pp = aux["proj_pairs"]
    raw_mimic = OL.mimic_feat_loss(pp[0], pp[1]) + OL.mimic_feat_loss(pp[2], pp[3])
    assert torch.allclose(r["recon"], raw_recon * lr * aux_w, rtol=1e-6)
    assert torch.allclose(r["mimic"], raw_mimic * lm * aux_w, rtol=1e-6)
    fn = sum(f.pow(2).mean() for f in aux["raw_feats"])
    want = (r["cls"] + fn * mp["lambda_feat_norm"] + mp["mask_parameters"]["lambda_mask"] * r["mask"]
            + lr * r["recon"] * aux_w + lm * r["mimic"] * aux_w)
    assert torch.allclose(r["total"], want, rtol=1e-6)
    # validation: hard labels, only the classification term, unweighted aux values
    assert torch.allclose(v["total"], OL.soft_weighted_focal(logits, y, mp["classification_loss_parameters"]["gamma"],
                                                             cw), rtol=1e-6)
    assert torch.allclose(v["recon"], raw_recon, rtol=1e-6)
