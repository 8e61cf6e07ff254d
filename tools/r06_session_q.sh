#!/bin/bash
# Round 6 final tree: mode-A kernel stats + conv-forward HBM traffic, then the mode-B weight-gradient traffic.
set -o pipefail
bash tools/modeA_prof.sh r06q > gpurun_out/r06q_a.txt 2>&1 || { echo "modeA prof failed"; tail -20 gpurun_out/r06q_a.txt; exit 1; }
bash tools/modeB_pmc.sh r06q_b > gpurun_out/r06q_b.txt 2>&1 || { echo "modeB pmc failed"; tail -20 gpurun_out/r06q_b.txt; exit 1; }
find gpurun_out -name '*.csv' -size +2M -exec gzip {} \;
du -sh gpurun_out
