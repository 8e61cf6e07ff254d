#!/usr/bin/env python3
"""Throughput benchmark of the DCE+DWI fusion training step on MI355X.

Metric (BASELINE.json): DCE+DWI volumes/sec/node (fwd+bwd). One volume = one
patient sample = a DWI stack [14,256,256] + a DCE stack [6,256,256]
(prepare_fusion_model.py:104-113). Workload = configuration 3 (fusion
classifier, batch 32 per GPU, S=256) in the reference's default training
state at epoch 0 ("mode A": both encoders frozen but in train mode -- dropout
on, BN batch statistics -- backward + AdamW through FusionModel only,
selector_helpers.py:437-443 / :632-685). ``--mode B`` unfreezes everything.

  python bench.py --gpus N --steps K --warmup W

--gpus N > 1 without a launcher's WORLD_SIZE starts N worker processes of this
script itself (one per GPU, RANK / LOCAL_RANK / WORLD_SIZE set, rendezvous on
127.0.0.1) before anything touches the GPU, and exits with their status; under
torch.distributed.run (WORLD_SIZE set) it is one of the ranks.

Prints ONE JSON line (rank 0) including the roofline of the dominant kernel
(the implicit-GEMM conv forward, timed per launch with HIP events on the
stream it runs on) and the CPU baseline (the fp32 CPU oracle restatement on a
bounded sample of the same workload).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "deep-multimodal-fusion-of-dce-mri-and-dwi-for-automated-breast-tumor-classification-w.-foundation_amd")
sys.path.insert(0, PKG)
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md chip table (spec)
BF16_MFMA_PEAK_TFLOPS = 2500.0  # dense bf16 (spec, no sparsity)
F32_MFMA_PEAK_TFLOPS = 157.3


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=None,
                    help="per-GPU batch (default 32; 16 for config 2, 4 for config 1)")
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--mode", choices=["A", "B"], default="A")
    ap.add_argument("--patch-embed", choices=["fp8", "bf16"], default="fp8",
                    help="config 5: PatchEmbed.proj on e4m3 MFMA (default) or the bf16 conv engine")
    ap.add_argument("--config", type=int, choices=[1, 2, 3, 5], default=3,
                    help="1: single-modality DWI CNN without backbone (C=16, S=128, train step); "
                         "2: DCE-only ResNet-50 OS8 feature extractor (5 phases, forward); "
                         "3: fusion step (default); "
                         "5: hybrid TransformerStage encoders (transformer_model.py, replaces block3), S=384 unless --size")
    ap.add_argument("--no-extras", action="store_true",
                    help="default run only: skip the mode-B, config-2 and config-5 sub-measurements")
    ap.add_argument("--dtype", choices=["bf16", "fp16", "fp32"], default="bf16",
                    help="compute dtype; fp16 = precision '16-mixed' (fp16 MFMA operands + dynamic loss scale)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--cpu-batch", type=int, default=32)
    ap.add_argument("--cpu-steps", type=int, default=3)
    ap.add_argument("--knob", action="append", default=[], metavar="NAME=VALUE",
                    help="flip a measured variant for an A/B run (dmf_ops.KNOBS; DESIGN.md 'Knobs')")
    return ap.parse_args()


def spawn_ranks(n):
    """``--gpus N`` with no launcher: N processes of this script, one per GPU,
    each with the torchrun environment (the parent never touches the GPU).
    Rank 0 prints the JSON line; the first failing rank stops the others."""
    import signal
    import socket
    import subprocess

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                for q in live:  # a rank died: the others would wait in a collective forever
                    q.send_signal(signal.SIGTERM)
        time.sleep(0.2)
    return rc


def build(P, device, dtype, mode, seed=0):
    import foundation_model as FM
    import model_module as MM
    import train_fusion as TF
    from selector_helpers import get_classification_loss

    torch.manual_seed(seed)
    P["dwi_model_parameters"]["compute_dtype"] = dtype
    if dtype == torch.float16:
        P["precision"] = "16-mixed"  # the reference's default: fp16 with dynamic loss scaling (DeviceGradScaler)
    P["backbone_freeze_on_start"] = mode == "A"
    bb_dwi = FM.build_medical_backbone(P, "cpu", "dwi", P["dwi_channel_num"])
    dwi = MM.initialize_model(MM.ModelMaskHeadBackbone("dwi", P, bb_dwi), True)
    bb_dce = FM.build_medical_backbone(P, "cpu", "dce", P["dce_channel_num"])
    dce = MM.initialize_model(MM.ModelMaskHeadBackbone("dce", P, bb_dce), True)
    fm = MM.FusionModel(P)
    dwi, dce, fm = dwi.to(device), dce.to(device), fm.to(device)
    train_labels = torch.arange(1024) % P["class_num"]  # balanced synthetic "train" labels -> weights ~1
    crit = get_classification_loss(P, train_labels, "fusion", device)
    lm = TF.LightningFusionModel(dwi, dce, fm, P, crit)
    lm.train()
    return lm


def synthetic_batch(B, S, device, seed, cd=14, cc=6):
    """DWI clamp(0.5+randn/6,0,1), DCE U[0,1), disc masks, labels randint(0,4)."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    dwi = (0.5 + torch.randn(B, cd, S, S, generator=g) / 6).clamp(0, 1)
    dce = torch.rand(B, cc, S, S, generator=g)
    yy, xx = torch.meshgrid(torch.arange(32), torch.arange(32), indexing="ij")
    masks = torch.zeros(B, 1, 32, 32)
    cyx = torch.randint(8, 24, (B, 2), generator=g)
    rad = torch.randint(4, 11, (B,), generator=g)
    for b in range(B):
        masks[b, 0] = (((yy - cyx[b, 0]) ** 2 + (xx - cyx[b, 1]) ** 2) <= rad[b] ** 2).float()
    labels = torch.randint(0, 4, (B,), generator=g)
    return tuple(t.to(device) for t in (dwi, dce, masks, labels))


# t_roof(fwd, B=32, bf16, S=256) = sum_k max(F_k / 2.5 PF, B_k / 8 TB/s)
# over the DWI + DCE encoder forward kernels (algorithmic F and B per kernel)
T_ROOF_ENC_FWD_MS_B32 = 2.69


def encoder_forward_probe(trainer, batch, args):
    """The north-star line: the fused DCE+DWI feature-extraction
    forward (both encoders, a1-a10, train-mode BN as in the step) timed alone
    from a hipGraph replay, against the survey's step roofline t_roof."""
    lm = trainer.lm
    dwi, dce = batch[0], batch[1]
    with torch.no_grad():
        for _ in range(2):
            lm._encode(dwi, dce)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            lm._encode(dwi, dce)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        with torch.cuda.graph(g):
            lm._encode(dwi, dce)
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 10
        e0.record()
        for _ in range(reps):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    out = {"ms": round(ms, 3), "volumes_per_s": round(args.batch / (ms * 1e-3), 1),
           "what": "DWI + DCE encoder forward (a1-a10), hipGraph replay, train-mode BN"}
    if args.config == 3 and args.size == 256 and args.dtype == "bf16":
        t_roof = T_ROOF_ENC_FWD_MS_B32 * args.batch / 32
        out.update({"t_roof_ms": round(t_roof, 3), "frac": round(t_roof / ms, 4),
                    "roof": "SURVEY 8(d): sum_k max(F_k / 2.5 PFLOP/s, B_k / 8 TB/s)"})
    return out


DT_TAG = {torch.bfloat16: "bf16", torch.float16: "f16", torch.float32: "f32"}


def mfma_peak(dtype):
    # the dense fp16 MFMA rate equals bf16's on gfx950
    return BF16_MFMA_PEAK_TFLOPS if dtype in (torch.bfloat16, torch.float16) else F32_MFMA_PEAK_TFLOPS


def wgrad_probe(trainer, batch, dtype):
    """Mode B's dominant kernel family, the MFMA weight gradient
    (k_conv_wgrad_dma / _tr + its split-K reduce): one eager mode-B step
    records every dmf_conv2d_wgrad + dmf_conv2d_wgrad_reduce pair; the pairs
    are replayed GPU-only from a hipGraph with HIP events around the replay
    (as roofline_probe). achieved = algorithmic 2*Cout*K*pixels per pair /
    average pair duration."""
    import dmf_ops as O

    recs = []
    O.PROBE["conv_wgrad"] = recs
    torch.cuda.synchronize()
    trainer.eager_step(batch)
    torch.cuda.synchronize()
    O.PROBE["conv_wgrad"] = None
    if not recs:
        return None
    flops = sum(r["flops"] for r in recs)
    byt = sum(r["bytes"] for r in recs)
    n = len(recs)
    avg_ms, per = O.probe_replay(recs)
    wg_only = [dict(r, calls=r["calls"][:1]) for r in recs]
    avg_ms_wg, _ = O.probe_replay(wg_only)
    recs.clear()
    peak = mfma_peak(dtype)
    achieved = flops / n / (avg_ms * 1e-3) / 1e12
    traffic = pmc_traffic("wgrad")
    return {"kernel": "conv2d weight gradient (k_conv_wgrad_dma / k_conv_wgrad_tr + k_wgrad_reduce), %s" %
                      DT_TAG[dtype],
            "bound": "mfma", "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
            "frac": round(achieved / peak, 4),
            "traffic": traffic["traffic_mb_per_launch"] if traffic else None,
            "traffic_unit": "MB per weight-gradient + split-reduce pair (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, " +
                            (traffic["source"] if traffic else "no PMC summary") + ")",
            "launches_per_step": n, "avg_launch_us": round(avg_ms * 1e3, 2),
            "avg_wgrad_kernel_us": round(avg_ms_wg * 1e3, 2),
            "avg_reduce_us": round((avg_ms - avg_ms_wg) * 1e3, 2),
            "algorithmic_gflop_per_launch": round(flops / n / 1e9, 3),
            "algorithmic_mb_per_launch": round(byt / n / 1e6, 2),
            "per_launch": "one launch = dmf_conv2d_wgrad + its dmf_conv2d_wgrad_reduce",
            **mfma_busy("mfma_wgrad", "wgrad")}


FP8_MFMA_PEAK_TFLOPS = 5000.0  # dense e4m3 (spec, no sparsity)


def gemm_probes(trainer, batch):
    """Config 5's rooflines: one eager step records the e4m3 patch-embed GEMM
    launches (dmf_gemm_fp8) and the bf16 token GEMMs (dmf_tokens.gemm:
    qkv / QK^T / PV / proj / fc1 / fc2), replayed GPU-only from a hipGraph
    (as roofline_probe); each family against its own dense MFMA peak."""
    import dmf_ops as O

    fam = {"fp8_gemm": ("e4m3 patch-embed GEMM (k_gemm_fp8_dma: 144x256 tiles, v_mfma_scale_f32_16x16x128_f8f6f4 "
                        "with unit scales; k_gemm_fp8 128x128 where those tiles do not fill the chip)",
                        FP8_MFMA_PEAK_TFLOPS),
           "tok_gemm": ("every token GEMM of the frozen encoders' blocks: qkv on the conv engine's persistent 1x1 "
                        "form, QK^T + PV inside the fused attention (dmf_flash_attn_fwd), fc1 (+ GELU + dropout) on "
                        "the conv engine, proj / fc2 on the conv engine's persistent 1x1 form with the LayerScale + "
                        "dropout + f32 residual register epilogue (dmf_conv2d_fwd_tokres); replayed at the tile sizing "
                        "they ran with inside the two-encoder fork", BF16_MFMA_PEAK_TFLOPS)}
    recs = {k: [] for k in fam}
    for k in fam:
        O.PROBE[k] = recs[k]
    torch.cuda.synchronize()
    try:
        trainer.eager_step(batch)
        torch.cuda.synchronize()
    finally:
        for k in fam:
            O.PROBE[k] = None
    out = {}
    for k, (name, peak) in fam.items():
        r = recs[k]
        if not r:
            continue
        n = len(r)
        # (the token family as recorded: proj / fc2's form exists only at the fork's half-chip sizing)
        avg_ms, per = O.probe_replay(r, as_recorded=k == "tok_gemm")
        flops = sum(x["flops"] for x in r)
        byt = sum(x["bytes"] for x in r)
        ach = flops / n / (avg_ms * 1e-3) / 1e12
        fl_of = {x["shape"]: x["flops"] for x in r}
        out[k] = {"kernel": name, "bound": "mfma", "achieved": round(ach, 2), "peak": peak, "unit": "TFLOP/s",
                  "frac": round(ach / peak, 4), "launches_per_step": n, "avg_launch_us": round(avg_ms * 1e3, 2),
                  "algorithmic_gflop_per_launch": round(flops / n / 1e9, 4),
                  "algorithmic_mb_per_launch": round(byt / n / 1e6, 3),
                  "per_shape": [{"shape": list(map(str, shp)), "launches": c, "us": round(t * 1e3, 2),
                                 "frac": round(fl_of[shp] / (t * 1e-3) / 1e12 / peak, 4)} for shp, c, t in per]}
        r.clear()
    return out


def roofline_probe(trainer, batch, dtype):
    """Average launch duration of the dominant kernel family (implicit-GEMM
    conv forward): one eager step records every conv-forward C-ABI launch
    (entry point, arguments, buffers); the recorded launches are then captured
    into a hipGraph and replayed on the stream they run on, with HIP events
    around the replay -- GPU time only, no host launch gaps."""
    import dmf_ops as O

    recs = []
    O.PROBE["conv_fwd"] = recs
    torch.cuda.synchronize()
    trainer.eager_step(batch)
    torch.cuda.synchronize()
    O.PROBE["conv_fwd"] = None
    if not recs:
        return None
    flops = sum(r["flops"] for r in recs)
    byt = sum(r["bytes"] for r in recs)
    n = len(recs)
    avg_ms, per = O.probe_replay(recs)
    ms = avg_ms * n
    dump = os.environ.get("DMF_CONV_DUMP")
    if dump:
        with open(dump, "w") as f:
            for shp, cnt, t in per:
                fl = next(r["flops"] for r in recs if r["shape"] == shp)
                for _ in range(cnt):
                    f.write(json.dumps({"shape": shp, "ms": round(t, 4), "gflop": round(fl / 1e9, 3),
                                        "tflops": round(fl / (t * 1e-3) / 1e12, 1)}) + "\n")
    recs.clear()
    peak = mfma_peak(dtype)
    achieved = flops / (ms * 1e-3) / 1e12
    traffic = pmc_traffic()
    return {
        "kernel": "conv2d forward (k_conv_fwd_ps / k_conv_fwd_pp / k_conv_fwd_sq / k_conv_fwd_wide / k_conv_fwd_buf / k_conv_stem / k_conv_igemm, %s)" %
                  DT_TAG[dtype],
        "bound": "mfma",
        "achieved": round(achieved, 2),
        "peak": peak,
        "unit": "TFLOP/s",
        "frac": round(achieved / peak, 4),
        "traffic": traffic["traffic_mb_per_launch"] if traffic else None,
        "traffic_unit": "MB per launch (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, " +
                        (traffic["source"] if traffic else "no PMC summary") + ")",
        "launches_per_step": n,
        "avg_launch_us": round(ms * 1e3 / n, 2),
        "algorithmic_gflop_per_launch": round(flops / n / 1e9, 3),
        "algorithmic_mb_per_launch": round(byt / n / 1e6, 2),
        "hbm_gbs_per_launch_avg": round(byt / (ms * 1e-3) / 1e9, 1),
        **mfma_busy("mfma", "conv_fwd"),
    }


PMC_LATEST = os.path.join(ROOT, "profiles", "pmc_latest.json")


def pmc_summary(key):
    """The PMC summary a committed pointer names: profiles/pmc_latest.json maps a
    key ("traffic" = conv forward HBM bytes, "traffic_wgrad", "mfma", "mfma_wgrad")
    to the summary file that tools/pmc_traffic.py / tools/pmc_mfma.py wrote for
    this tree (--latest KEY updates the pointer). The pointer is data in the
    repo, so a fresh clone reads the same file whatever the checkout's mtimes."""
    try:
        with open(PMC_LATEST) as f:
            rel = json.load(f).get(key)
    except (OSError, ValueError):
        return None
    if not rel:
        return None
    path = os.path.join(ROOT, rel)
    if not os.path.exists(path):
        return None
    with open(path) as f:
        d = json.load(f)
    d["source"] = rel
    return d


def mfma_busy(key, form):
    """MFMA utilisation of a kernel family from the committed counter summary (tools/pmc_mfma.py:
    SQ_VALU_MFMA_BUSY_CYCLES / (4 SIMDs x CUs x GRBM_GUI_ACTIVE/8), PMC passes serialise dispatches)."""
    d = pmc_summary(key)
    row = (d or {}).get("forms", {}).get(form)
    if not row:
        return {"mfma_busy": None}
    return {"mfma_busy": row["mfma_busy_cu"], "mfma_busy_chip": row["mfma_busy_chip"],
            "mfma_busy_unit": "SQ_VALU_MFMA_BUSY_CYCLES / (4 x occupied CUs x GRBM_GUI_ACTIVE/8) over the family's "
                              "dispatches (chip: over all 256 CUs), " + d["source"]}


def pmc_traffic(family=""):
    """HBM bytes per launch of a kernel family (FETCH_SIZE x2 + WRITE_SIZE from
    two rocprofv3 --pmc passes of this bench on an MI355X; tools/pmc_traffic.py)."""
    return pmc_summary("traffic_" + family if family else "traffic")


def _cpu_params(PR, args):
    P = PR.default_parameters()
    if args.config == 5:
        P["dwi_model_parameters"]["use_hybrid_transformer"] = True
    P["dwi_model_parameters"]["input_size"] = args.size
    return P


def cpu_threads():
    """Host threads for the CPU baseline: the process's CPU share. On the GPU
    box os.cpu_count() reports the whole machine while OMP_NUM_THREADS holds
    this job's share (16), so the share wins when it is set."""
    env = os.environ.get("OMP_NUM_THREADS")
    n = int(env) if env and env.isdigit() and int(env) > 0 else (os.cpu_count() or 1)
    try:
        n = min(n, len(os.sched_getaffinity(0)))
    except AttributeError:
        pass
    return max(1, n)


def cpu_baseline(args, P_fn):
    """fp32 CPU oracle (same eager op sequence as the reference) on a bounded
    sample of the benched workload: cpu-batch volumes at SxS (B=32 = the GPU
    line's per-GPU batch), mode A/B step, 1 warm-up then the median of
    cpu-steps timed steps (3 timed steps after 1 warm-up)."""
    from oracle import losses as OL
    from oracle import model as OM

    torch.set_num_threads(cpu_threads())
    P = P_fn()
    P["dwi_model_parameters"]["backbone_index_lists"] = [[0], [1], [2, 3]]
    torch.manual_seed(0)
    dwi = OM.ModelMaskHeadBackbone("dwi", P, OM.ResNet50OS8(P["dwi_channel_num"]))
    dce = OM.ModelMaskHeadBackbone("dce", P, OM.ResNet50OS8(P["dce_channel_num"]))
    fm = OM.FusionModel(P)
    for m in (dwi, dce):
        for p in m.parameters():
            p.requires_grad = (args.mode == "B")
    params = [p for m in (dwi, dce, fm) for p in m.parameters() if p.requires_grad]
    opt = torch.optim.AdamW(params, lr=1e-4, weight_decay=1e-4)
    b = synthetic_batch(args.cpu_batch, args.size, "cpu", 1)
    cw = OL.class_weights_from_labels(torch.arange(1024) % 4)

    def step():
        opt.zero_grad()
        out = OL.fusion_shared_step(dwi, dce, fm, b, P, cw, epoch=0)
        out["total"].backward()
        opt.step()

    step()
    times = []
    for _ in range(args.cpu_steps):
        t0 = time.perf_counter()
        step()
        times.append(time.perf_counter() - t0)
    med = sorted(times)[len(times) // 2]
    return {"value": round(args.cpu_batch / med, 4), "unit": "volumes/s",
            "cores": torch.get_num_threads(), "host_cpu_count": os.cpu_count(), "kind": "port",
            "step_s": [round(t, 3) for t in times],
            "sample": f"oracle fp32 CPU (torch eager, {torch.get_num_threads()} threads = this job's CPU share; "
                      f"os.cpu_count() {os.cpu_count()}), config {args.config} mode {args.mode}, median of "
                      f"{args.cpu_steps} timed steps x {args.cpu_batch} volumes at {args.size}x{args.size} "
                      f"(1 warm-up step)"}


def cpu_baseline_mode_b(args, P_fn, batch=4, steps=2):
    """BASELINE.md's mode-B CPU line: the fp32 oracle's mode-B step (every
    encoder parameter trainable) on a bounded sample -- `batch` volumes at SxS,
    1 warm-up then the median of `steps` timed steps (a B=32 mode-B CPU step
    runs ~20 s; the sample keeps the default bench within minutes)."""
    import copy
    a = copy.copy(args)
    a.mode, a.cpu_batch, a.cpu_steps = "B", batch, steps
    out = cpu_baseline(a, P_fn)
    out["sample"] = out["sample"].replace("mode B", "mode B (all trainable)")
    return out


def cpu_baseline_config1(batch=4, size=128, chans=16, steps=2):
    """BASELINE.md's config-1 CPU line (config 1 IS the reference's CPU case:
    'CPU PyTorch, train.py one epoch'): the oracle's single-modality DWI CNN
    training step (use_backbone=False, C=16, S=128, B=4; oracle.losses.
    single_shared_step = train.py:294-466) + torch AdamW, fp32, 1 warm-up then
    the median of `steps` timed steps."""
    import parameters as PR
    from oracle import losses as OL
    from oracle import model as OM

    torch.set_num_threads(cpu_threads())
    P = PR.default_parameters()
    mp = P["dwi_model_parameters"]
    mp["use_backbone"] = False
    mp["input_size"] = size
    P["dwi_channel_num"] = chans
    torch.manual_seed(0)
    ref = OM.ModelMaskHeadBackbone("dwi", P, None)
    ref.train()
    opt = torch.optim.AdamW(ref.parameters(), lr=1e-4, weight_decay=4e-5)
    g = torch.Generator().manual_seed(0)
    x = (0.5 + torch.randn(batch, chans, size, size, generator=g) / 6).clamp(0, 1)
    masks = (torch.rand(batch, 1, 32, 32, generator=g) > 0.5).float()
    labels = torch.arange(batch) % 4
    cw = OL.class_weights_from_labels(torch.arange(1024) % 4)

    def step():
        opt.zero_grad()
        OL.single_shared_step(ref, (x, masks, labels), P, cw, "dwi", epoch=0)["total"].backward()
        opt.step()

    step()
    times = []
    for _ in range(steps):
        t0 = time.perf_counter()
        step()
        times.append(time.perf_counter() - t0)
    med = sorted(times)[len(times) // 2]
    return {"value": round(batch / med, 3), "unit": "volumes/s", "cores": torch.get_num_threads(),
            "host_cpu_count": os.cpu_count(), "kind": "port", "step_s": [round(t, 3) for t in times],
            "sample": f"oracle fp32 CPU, config 1 (DWI CNN, use_backbone=False, C={chans}, S={size}, B={batch}) "
                      f"training step + AdamW, median of {steps} timed steps (1 warm-up)"}


def _graph(fn):
    """Capture fn() (GPU work only, inputs resident) into a hipGraph after
    two eager runs on a side stream (allocator / weight-cache warm-up)."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = fn()
    return g, out


def _median_step_ms(step, n):
    """Median of n individually event-timed steps (SURVEY 8(d) timing
    procedure) -- reported beside the pipelined K-step mean."""
    evs = []
    for _ in range(n):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        step()
        e1.record()
        evs.append((e0, e1))
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) for a, b in evs)
    return ts[len(ts) // 2]


def conv_probe(fn, dtype):
    """Dominant-kernel roofline of one eager run of fn (see roofline_probe)."""
    import dmf_ops as O

    recs = []
    O.PROBE["conv_fwd"] = recs
    torch.cuda.synchronize()
    fn()
    torch.cuda.synchronize()
    O.PROBE["conv_fwd"] = None
    if not recs:
        return None
    flops = sum(r["flops"] for r in recs)
    byt = sum(r["bytes"] for r in recs)
    n = len(recs)
    avg_ms, _ = O.probe_replay(recs)
    peak = mfma_peak(dtype)
    achieved = flops / n / (avg_ms * 1e-3) / 1e12
    recs.clear()
    return {"kernel": "conv2d forward (k_conv_fwd_ps / k_conv_fwd_pp / k_conv_fwd_sq / k_conv_fwd_wide / k_conv_fwd_buf / k_conv_stem / k_conv_igemm)",
            "bound": "mfma", "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
            "frac": round(achieved / peak, 4), "traffic": None, "launches_per_step": n,
            "avg_launch_us": round(avg_ms * 1e3, 2), "algorithmic_gflop_per_launch": round(flops / n / 1e9, 3),
            "algorithmic_mb_per_launch": round(byt / n / 1e6, 2)}


# timm ResNet-50 OS8, in_chans=5, S=256: 50.0 GFLOP per volume (2 x MACs of every conv)
CONFIG2_GFLOP_PER_VOL = 50.0


def bench_config2(device, batch, steps, warmup, size=256, probe=True):
    """Config 2: DCE-only foundation feature extractor (foundation_model.py:
    build_medical_backbone(..., 'dce', in_channels=5) -> timm resnet50
    features_only OS8, :260-267), bf16, forward only, inference (eval BN),
    inputs resident in HBM; one step = one forward over the batch, replayed
    from a hipGraph."""
    import foundation_model as FM
    import parameters as PR

    P = PR.default_parameters()
    P["dce_channel_num"] = 5
    P["dwi_model_parameters"]["compute_dtype"] = torch.bfloat16
    torch.manual_seed(0)
    bb = FM.build_medical_backbone(P, "cpu", "dce", 5).to(device).eval()
    for p in bb.parameters():
        p.requires_grad = False
    g = torch.Generator().manual_seed(1)
    x = torch.rand(batch, 5, size, size, generator=g).to(device)

    def fwd():
        with torch.no_grad():
            return bb(x)

    graph, feats = _graph(fwd)
    for _ in range(warmup):
        graph.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        graph.replay()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ms = dt * 1e3 / steps
    med = _median_step_ms(graph.replay, max(5, min(steps, 50)))
    gflop = CONFIG2_GFLOP_PER_VOL * (size / 256) ** 2
    tf = gflop * batch / (ms * 1e-3) / 1e3
    finite = all(bool(torch.isfinite(f).all()) for f in feats)
    out = {"metric": "DCE volumes/sec (foundation feature extraction, fwd)", "value": round(batch * steps / dt, 2),
           "unit": "volumes/s", "ms_per_step": round(ms, 3), "ms_per_step_median": round(med, 3),
           "steps": steps, "warmup": warmup, "dtype": "bf16", "finite": finite,
           "config": {"workload": "config 2: DCE-only ResNet-50 OS8 feature extractor (5 phases, eval BN, fwd)",
                      "per_gpu_batch": batch, "size": size, "in_chans": 5, "hipgraph": True},
           "step_roofline": {"bound": "mfma", "achieved": round(tf, 1), "peak": BF16_MFMA_PEAK_TFLOPS,
                             "unit": "TFLOP/s", "frac": round(tf / BF16_MFMA_PEAK_TFLOPS, 4),
                             "algorithmic_gflop_per_volume": gflop}}
    if probe:
        out["roofline"] = conv_probe(fwd, torch.bfloat16)
    del graph
    return out


def bench_config1(device, batch, steps, warmup, size=128, chans=16):
    """Config 1: the single-modality DWI CNN without backbone
    (model_module.py:550-552, :663-666), C=16, S=128, one training step =
    LightningSingleModel.training_step -> backward -> AdamW (train.py:294-428),
    bf16, replayed from a hipGraph."""
    import model_module as MM
    import parameters as PR
    import train as TR
    from dmf_optim import FusedAdamW
    from selector_helpers import get_classification_loss

    P = PR.default_parameters()
    mp = P["dwi_model_parameters"]
    mp["use_backbone"] = False
    mp["input_size"] = size
    mp["compute_dtype"] = torch.bfloat16
    P["dwi_channel_num"] = chans
    torch.manual_seed(0)
    enc = MM.initialize_model(MM.ModelMaskHeadBackbone("dwi", P, None), True).to(device)
    crit = get_classification_loss(P, torch.arange(1024) % P["class_num"], "dwi", device)
    lm = TR.LightningSingleModel(model=enc, method="dwi", criterion_clf=crit, parameters_dict=P)
    lm.train()
    opt = FusedAdamW(lm.parameters(), lr=1e-4, weight_decay=4e-5)
    g = torch.Generator().manual_seed(0)
    x = (0.5 + torch.randn(batch, chans, size, size, generator=g) / 6).clamp(0, 1).to(device)
    masks = (torch.rand(batch, 1, 32, 32, generator=g) > 0.5).float().to(device)
    labels = (torch.arange(batch) % 4).to(device)

    def step():
        opt.zero_grad(set_to_none=False)
        loss = lm.training_step((x, masks, labels))
        loss.backward()
        opt.step()
        return loss.detach()

    step()  # the optimizer's tables exist before capture
    graph, loss = _graph(step)
    for _ in range(warmup):
        graph.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        graph.replay()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return {"metric": "DWI volumes/sec (single-modality CNN training step, fwd+bwd+AdamW)",
            "value": round(batch * steps / dt, 2), "unit": "volumes/s", "ms_per_step": round(dt * 1e3 / steps, 3),
            "steps": steps, "warmup": warmup, "dtype": "bf16", "loss": round(float(loss.item()), 5),
            "config": {"workload": "config 1: DWI CNN, use_backbone=False, all trainable", "per_gpu_batch": batch,
                       "size": size, "in_chans": chans, "hipgraph": True}}


def bench_fusion(P, device, dtype, mode, batch_size, size, steps, warmup, world, rank, use_graph=True):
    """Config 3/5 fusion training step -> (trainer, batch, seconds for steps)."""
    from dmf_dp import FusionTrainer

    lm = build(P, device, dtype, mode, seed=0)
    trainer = FusionTrainer(lm, world=world, use_graph=use_graph)
    batch = synthetic_batch(batch_size, size, device, seed=2 + rank)
    if use_graph:
        trainer.capture(batch)
    for _ in range(warmup):
        trainer.step(batch)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        trainer.step(batch)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = t.item()
    return trainer, batch, dt


# algorithmic work per volume of the fusion step
GFLOP_PER_VOL = {"A": 155.0, "B": 458.0}


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # the parent never touches HIP (no device query either): each rank checks its own cuda:<rank>
        assert not torch.cuda.is_initialized(), "bench.py parent initialised HIP before spawning ranks"
        sys.exit(spawn_ranks(args.gpus))
    rank, local_rank, world = int(os.environ.get("RANK", 0)), int(os.environ.get("LOCAL_RANK", 0)), \
        int(os.environ.get("WORLD_SIZE", 1))
    if world != args.gpus and rank == 0:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE {world}; measuring {world} rank(s)", file=sys.stderr)
    # one process per GPU over RCCL ("nccl"). DMF_DIST_BACKEND=gloo with
    # DMF_BENCH_SHARE_GPU=1 rehearses the multi-rank control flow on a 1-GPU box.
    ndev = torch.cuda.device_count()
    if os.environ.get("DMF_BENCH_SHARE_GPU") == "1" and ndev > 0:
        dev_idx = local_rank % ndev
    else:
        dev_idx = local_rank
        if dev_idx >= ndev:
            print(f"bench.py rank {rank}: cuda:{dev_idx} is not visible ({ndev} GPU(s)); "
                  f"--gpus {args.gpus} needs one GPU per rank", file=sys.stderr, flush=True)
            sys.exit(3)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(dev_idx)
        backend = os.environ.get("DMF_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_idx))
        else:
            dist.init_process_group(backend)
    device = torch.device("cuda", dev_idx)
    import parameters as PR

    if args.knob:
        import dmf_ops as O

        O.set_knobs(**dict(k.split("=", 1) for k in args.knob))

    if args.config in (1, 2):
        if world > 1:
            raise SystemExit("configs 1 and 2 are single-GPU configurations (BASELINE.json)")
        if args.config == 2:
            out = bench_config2(device, args.batch or 16, args.steps, args.warmup,
                                size=args.size, probe=not args.no_roofline)
        else:
            out = bench_config1(device, args.batch or 4, args.steps, args.warmup,
                                size=128 if args.size == 256 else args.size)
        out.update({"n_gpus": 1, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
                    "data": "synthetic volumes, random-init weights"})
        if args.config == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline_config1(batch=args.batch or 4)
        print(json.dumps(out), flush=True)
        return

    args.batch = args.batch or 32
    dtype = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}[args.dtype]
    P = PR.default_parameters()
    if args.config == 5:
        # hybrid CNN -> Transformer stage (E=512, depth 6, 4 heads, patch 2;
        # parameters_generate.py:71-75) in place of block3, S=384 (576 tokens per volume)
        P["dwi_model_parameters"]["use_hybrid_transformer"] = True
        # config 5 names an fp8-e4m3 MFMA patch-embed (bf16 elsewhere)
        P["dwi_model_parameters"]["patch_embed_fp8"] = args.patch_embed == "fp8" and dtype == torch.bfloat16
        if args.size == 256:
            args.size = 384
    P["dwi_model_parameters"]["input_size"] = args.size
    trainer, batch, dt = bench_fusion(P, device, dtype, args.mode, args.batch, args.size, args.steps, args.warmup,
                                      world, rank, use_graph=not args.no_graph)
    loss_val = float(trainer.loss.item()) if trainer.loss is not None else None
    comm_ranks = trainer._rccl.count() if getattr(trainer, "_rccl", None) is not None else None
    if loss_val is not None and loss_val != loss_val:
        raise RuntimeError("training loss is NaN: the benchmarked step is numerically broken")
    med = _median_step_ms(lambda: trainer.step(batch), min(args.steps, 50)) if world == 1 else None
    roof = None
    if not args.no_roofline:
        # every rank: the probe's eager step contains the gradient all-reduce
        roof = roofline_probe(trainer, batch, dtype)
    enc = encoder_forward_probe(trainer, batch, args) if (rank == 0 and not args.no_roofline) else None

    vols = args.batch * world * args.steps
    ms = dt * 1e3 / args.steps
    out = {
        "metric": "DCE+DWI volumes/sec/node (fwd+bwd)",
        "value": round(vols / dt, 2),
        "unit": "volumes/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 3),
        "ms_per_step_median": round(med, 3) if med is not None else None,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": "synthetic (config-3 recipe: DWI clamp(0.5+N/6), DCE U[0,1), disc masks); random-init weights",
        "config": {"workload": f"fusion training step, config {args.config}, mode {args.mode} "
                               f"({'encoders frozen, train-mode' if args.mode == 'A' else 'all trainable'})",
                   "global_batch": args.batch * world, "per_gpu_batch": args.batch, "size": args.size,
                   "parallelism": f"dp{world}", "hipgraph": not args.no_graph,
                   "collective": ("RCCL all-reduce over %d ranks (ncclCommCount), overlapped with backward" % comm_ranks
                                  if comm_ranks else ("gloo host all-reduce" if world > 1 else "none (1 rank)")),
                   **({"patch_embed": args.patch_embed if args.dtype == "bf16" else "f32"}
                      if args.config == 5 else {})},
        "loss": loss_val,
        "peak_hbm_gb": round(torch.cuda.max_memory_allocated(device) / 2**30, 2),
        "roofline": roof,
    }
    if args.config == 3 and args.size == 256:
        tf = GFLOP_PER_VOL[args.mode] * args.batch / (ms * 1e-3) / 1e3
        out["step_roofline"] = {"bound": "mfma", "achieved": round(tf, 1), "peak": BF16_MFMA_PEAK_TFLOPS,
                                "unit": "TFLOP/s", "frac": round(tf / BF16_MFMA_PEAK_TFLOPS, 4),
                                "algorithmic_gflop_per_volume": GFLOP_PER_VOL[args.mode]}
    if enc is not None:
        out["encoder_forward"] = enc
    extras = (args.config == 3 and args.mode == "A" and args.dtype == "bf16" and args.size == 256
              and not args.no_extras)
    del trainer
    if extras:
        # mode B (all unfrozen) is the DP-scaling headline; measured on every rank (it is a
        # second fusion step, same exchange), reported by rank 0
        torch.cuda.empty_cache()
        tb, bb_, dtb = bench_fusion(PR.default_parameters(), device, dtype, "B", args.batch, args.size,
                                    max(10, args.steps // 2), 3, world, rank, use_graph=not args.no_graph)
        nb = max(10, args.steps // 2)
        msb = dtb * 1e3 / nb
        roof_b = wgrad_probe(tb, bb_, dtype) if not args.no_roofline else None
        tfb = GFLOP_PER_VOL["B"] * args.batch / (msb * 1e-3) / 1e3
        out["mode_b"] = {"value": round(args.batch * world * nb / dtb, 2), "unit": "volumes/s",
                         "ms_per_step": round(msb, 3), "steps": nb, "warmup": 3,
                         "loss": float(tb.loss.item()) if tb.loss is not None else None,
                         "workload": "fusion training step, config 3, mode B (all trainable)",
                         "step_roofline": {"bound": "mfma", "achieved": round(tfb, 1),
                                           "peak": BF16_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                                           "frac": round(tfb / BF16_MFMA_PEAK_TFLOPS, 4),
                                           "algorithmic_gflop_per_volume": GFLOP_PER_VOL["B"]},
                         "roofline": roof_b}
        del tb, bb_
        torch.cuda.empty_cache()
        if world == 1:
            out["config2"] = bench_config2(device, 16, 20, 5, probe=False)
        # hybrid TransformerStage encoders at S=384 (576 tokens, E=512, depth 6,
        # 4 heads; parameters_generate.py:71-75) with the fp8-e4m3 MFMA patch-embed, bf16 elsewhere,
        # mode A, B=32 per GPU -- a DP configuration, so measured on every rank like mode B
        torch.cuda.empty_cache()
        P5 = PR.default_parameters()
        P5["dwi_model_parameters"]["use_hybrid_transformer"] = True
        P5["dwi_model_parameters"]["patch_embed_fp8"] = True
        P5["dwi_model_parameters"]["input_size"] = 384
        n5 = max(10, args.steps // 2)
        t5, b5, dt5 = bench_fusion(P5, device, dtype, "A", args.batch, 384, n5, 3, world, rank,
                                   use_graph=not args.no_graph)
        roof5 = gemm_probes(t5, b5) if not args.no_roofline else None
        out["config5"] = {"value": round(args.batch * world * n5 / dt5, 2), "unit": "volumes/s",
                          "ms_per_step": round(dt5 * 1e3 / n5, 3), "steps": n5, "warmup": 3,
                          "loss": float(t5.loss.item()) if t5.loss is not None else None,
                          "workload": "fusion training step, config 5 (hybrid TransformerStage encoders, S=384, "
                                      "fp8-e4m3 patch-embed, bf16 elsewhere), mode A",
                          "per_gpu_batch": args.batch, "size": 384, "patch_embed": "fp8",
                          "roofline": roof5}
        del t5, b5
        torch.cuda.empty_cache()
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            out["cpu_baseline"] = cpu_baseline(args, lambda: _cpu_params(PR, args))
        except Exception as e:  # report, never hide
            out["cpu_baseline"] = {"error": repr(e)}
        if extras:
            # CPU volumes/s for config 1 (B=4) and config 3 modes A and B
            for key, fn in (("cpu_baseline_mode_b", lambda: cpu_baseline_mode_b(args, lambda: _cpu_params(PR, args))),
                            ("cpu_baseline_config1", cpu_baseline_config1)):
                try:
                    out[key] = fn()
                except Exception as e:
                    out[key] = {"error": repr(e)}
            if "mode_b" in out and "value" in out.get("cpu_baseline_mode_b", {}):
                out["mode_b"]["cpu_baseline"] = out["cpu_baseline_mode_b"]
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
