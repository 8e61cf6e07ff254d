#!/bin/bash
# r05v: half-chip dgrad tiles in a two-encoder backward (knob conc_bwd_min_tiles), mode-B A/B.
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  for v in 128 0; do
    timeout -k 10 200 python bench.py --mode B --no-extras --no-cpu-baseline --no-roofline --steps 25 --warmup 5 --knob conc_bwd_min_tiles=$v > gpurun_out/r05v_modeB_conc$v.$i.json 2> gpurun_out/r05v_modeB_conc$v.$i.err || { echo "bench rc=$?"; tail -5 gpurun_out/r05v_modeB_conc$v.$i.err; exit 1; }
    echo "conc_bwd_min_tiles=$v round $i: $(cut -c1-140 gpurun_out/r05v_modeB_conc$v.$i.json)"
  done
done
