#!/bin/bash
# Interleaved per-shape A/B of library variants ab/<name>.so on tools/conv_bench.py (BN statistics into the
# float64 arena, as the training forward): usage: bash tools/lib_conv_ab.sh ROUNDS "ONLY" name1 name2 ...
set -o pipefail
R=${1:?rounds}; ONLY=${2:?shape indices}; shift 2
mkdir -p gpurun_out/libab
for r in $(seq 1 $R); do
  for n in "$@"; do
    echo "== $n round $r"
    DMF_HIP_LIB=ab/$n.so timeout -k 10 200 python tools/conv_bench.py --acc --only "$ONLY" --reps 20 2>gpurun_out/libab/$n.$r.err || { echo "conv_bench $n failed"; tail -20 gpurun_out/libab/$n.$r.err; exit 1; }
  done
done
