#!/bin/bash
# r05n: the XCD split-major weight-gradient order: per-shape A/B (tools/wgrad_bench.py --xcd), the
# kernel tests of the weight gradient with it on, then the mode-B step A/B (interleaved bench runs).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/wgrad_bench.py --xcd --from profiles/r04f_conv_launches.jsonl --rounds 3 > gpurun_out/r05n_wgrad_xcd.txt 2>&1 || { echo "wgrad_bench rc=$?"; tail -5 gpurun_out/r05n_wgrad_xcd.txt; exit 1; }
tail -3 gpurun_out/r05n_wgrad_xcd.txt
for i in 1 2; do
  for v in 0 1; do
    timeout -k 10 200 python bench.py --mode B --no-extras --no-cpu-baseline --no-roofline --steps 25 --warmup 5 --knob wgrad_xcd=$v > gpurun_out/r05n_modeB_xcd$v.$i.json 2> gpurun_out/r05n_modeB_xcd$v.$i.err || { echo "bench rc=$?"; tail -5 gpurun_out/r05n_modeB_xcd$v.$i.err; exit 1; }
    echo "xcd=$v round $i: $(cut -c1-160 gpurun_out/r05n_modeB_xcd$v.$i.json)"
  done
done
