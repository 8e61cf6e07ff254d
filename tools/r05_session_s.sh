#!/bin/bash
# r05s: half-chip 256-wide forward tiles inside the two-encoder fork (knob conc_min_tiles), mode-A A/B.
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  for v in 128 0; do
    timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline --no-roofline --steps 50 --warmup 10 --knob conc_min_tiles=$v > gpurun_out/r05s_modeA_conc$v.$i.json 2> gpurun_out/r05s_modeA_conc$v.$i.err || { echo "bench rc=$?"; tail -5 gpurun_out/r05s_modeA_conc$v.$i.err; exit 1; }
    echo "conc_min_tiles=$v round $i: $(cut -c1-140 gpurun_out/r05s_modeA_conc$v.$i.json)"
  done
done
timeout -k 10 300 python -u tools/enc_fwd_ab.py --tunes "conc_min_tiles=128;conc_min_tiles=0" --rounds 5 > gpurun_out/r05s_enc_ab.txt 2>&1 || exit 1
tail -2 gpurun_out/r05s_enc_ab.txt
