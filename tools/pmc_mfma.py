#!/usr/bin/env python3
"""MFMA utilisation and LDS behaviour per conv form from two rocprofv3 --pmc
passes of the bench step (tools/pmc_mfma.sh writes them):

  pass sq : SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY
            SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS
            SQ_INSTS_LDS + GRBM_GUI_ACTIVE
  pass lds: SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU
            + GRBM_GUI_ACTIVE

Units (MI355X_MICROARCH.md, "s_memtime tick vs SQ PMC units" and "DVFS
give-back"): SQ_VALU_MFMA_BUSY_CYCLES counts busy cycles summed over every
SIMD (16 per 16x16x32 bf16 MFMA); GRBM_GUI_ACTIVE is summed over the 8 XCDs,
so one dispatch lasts GRBM_GUI_ACTIVE / 8 shader cycles; SQ_WAVE_CYCLES and
the SQ_WAIT_* / SQ_ACTIVE_* counters count quad-cycles (ratios between them
are unit-free). PMC collection serialises dispatches, so each figure is the
dispatch running alone.

  mfma_busy_chip = MFMA_BUSY / (4 SIMDs x 256 CUs x GRBM_GUI_ACTIVE / 8)
  mfma_busy_cu   = the same over the CUs the dispatch occupies
                   (min(blocks, 256) for the one-block-per-CU 256-wide forms)

usage: pmc_mfma.py DIR [--json OUT] [--latest KEY]
"""
import argparse
import collections
import csv
import glob
import json
import os
import re
import sys

NCU = 256
FORMS = [
    ("pp", r"k_conv_fwd_pp<"), ("ps", r"k_conv_fwd_ps<"), ("sq", r"k_conv_fwd_sq<"),
    ("wide", r"k_conv_fwd_wide<"), ("buf", r"k_conv_fwd_buf<"), ("stem", r"k_conv_stem<"),
    ("igemm", r"k_conv_igemm<unsigned short, false"),
    ("wgrad", r"k_conv_wgrad_(dma|tr)<"), ("wgrad_reduce", r"k_wgrad_reduce"),
    ("bn_apply", r"k_bn_apply<"),
]
ONE_BLOCK_PER_CU = {"pp", "ps", "sq", "wide", "wgrad"}


def load(d):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        sys.exit("no counter_collection.csv under " + d)
    disp = collections.defaultdict(dict)
    meta = {}
    for r in csv.DictReader(open(f[0])):
        key = r["Dispatch_Id"]
        disp[key][r["Counter_Name"]] = disp[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        meta[key] = (r["Kernel_Name"], int(r["Grid_Size"]) // max(1, int(r["Workgroup_Size"])))
    return disp, meta


def form_of(name):
    for f, rx in FORMS:
        if re.search(rx, name):
            return f
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--json", default="")
    ap.add_argument("--latest", default="")
    ap.add_argument("--by-kernel", action="store_true", help="also one row per kernel template instance")
    a = ap.parse_args()
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for sub in ("sq", "lds"):
        path = os.path.join(a.dir, sub)
        if not os.path.isdir(path):
            continue
        disp, meta = load(path)
        for k, cs in disp.items():
            name, blocks = meta[k]
            f = form_of(name)
            if f is None:
                continue
            groups = [f] + ([name[:100]] if a.by_kernel else []) + (["conv_fwd"] if f not in (
                "wgrad", "wgrad_reduce", "bn_apply") else [])
            cyc = cs.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
            cus = min(blocks, NCU) if f in ONE_BLOCK_PER_CU else NCU
            for g in groups:
                A = agg[g]
                A[sub + "_n"] += 1
                for c, v in cs.items():
                    A[sub + ":" + c] += v
                A[sub + ":cyc"] += cyc
                A[sub + ":cu_cyc"] += cyc * cus
    out = {}
    for g, A in sorted(agg.items(), key=lambda kv: -kv[1].get("sq:cyc", 0.0)):
        n = int(A.get("sq_n", 0))
        if not n:
            continue
        busy = A.get("sq:SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        wave = A.get("sq:SQ_WAVE_CYCLES", 0.0) or 1.0
        row = {
            "dispatches": n,
            "avg_us_at_2.1GHz": round(A["sq:cyc"] / n / 2100.0, 2),
            "mfma_busy_chip": round(busy / (4 * NCU * A["sq:cyc"]), 4) if A["sq:cyc"] else None,
            "mfma_busy_cu": round(busy / (4 * A["sq:cu_cyc"]), 4) if A["sq:cu_cyc"] else None,
            "wait_any_of_wave": round(A.get("sq:SQ_WAIT_ANY", 0.0) / wave, 4),
            "wait_inst_any_of_wave": round(A.get("sq:SQ_WAIT_INST_ANY", 0.0) / wave, 4),
            "wait_inst_lds_of_wave": round(A.get("sq:SQ_WAIT_INST_LDS", 0.0) / wave, 4),
            "active_inst_of_wave": round(A.get("sq:SQ_ACTIVE_INST_ANY", 0.0) / wave, 4),
            "lds_insts_per_dispatch": round(A.get("sq:SQ_INSTS_LDS", 0.0) / n, 1),
        }
        nl = int(A.get("lds_n", 0))
        if nl:
            idx = A.get("lds:SQ_LDS_IDX_ACTIVE", 0.0)
            row["lds_bank_conflict_of_active"] = round(A.get("lds:SQ_LDS_BANK_CONFLICT", 0.0) / idx, 4) if idx else None
            row["lds_active_of_cu_cycles"] = round(idx / A["lds:cu_cyc"], 4) if A.get("lds:cu_cyc") else None
            row["valu_insts_per_dispatch"] = round(A.get("lds:SQ_INSTS_VALU", 0.0) / nl, 1)
        out[g] = row
        print(f"{g[:60]:60s} " + " ".join(f"{k}={v}" for k, v in row.items()))
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"source": a.dir, "ncu": NCU, "forms": out,
                       "definition": "mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (4 x CUs x GRBM_GUI_ACTIVE/8); "
                                     "PMC passes serialise dispatches"}, f, indent=1)
        if a.latest:
            sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
            from pmc_traffic import set_latest
            set_latest(a.latest, a.json)


if __name__ == "__main__":
    main()
