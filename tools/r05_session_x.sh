#!/bin/bash
# r05x: two-pass K threshold under the two-stream tile sizing; mode-B weight-gradient fill.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/enc_fwd_ab.py --tunes "two_pass_max_k=256;two_pass_max_k=512;two_pass_max_k=128" --rounds 5 > gpurun_out/r05x_twopass_k_ab.txt 2>&1 || exit 1
grep variant gpurun_out/r05x_twopass_k_ab.txt
for i in 1 2; do
  for v in 50 100 25; do
    timeout -k 10 200 python bench.py --mode B --no-extras --no-cpu-baseline --no-roofline --steps 25 --warmup 5 --knob wgrad_fill=$v > gpurun_out/r05x_modeB_fill$v.$i.json 2> gpurun_out/r05x_modeB_fill$v.$i.err || { echo "bench rc=$?"; tail -5 gpurun_out/r05x_modeB_fill$v.$i.err; exit 1; }
    echo "wgrad_fill=$v round $i: $(cut -c1-140 gpurun_out/r05x_modeB_fill$v.$i.json)"
  done
done
