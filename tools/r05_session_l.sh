#!/bin/bash
# r05l: config-5 fusion-stage errors, the flash-attention bench after the Philox change, the mode-B PMC
# traffic passes. Each GPU step under its own limit; a non-zero status ends the script.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/config5_stage_errors.py --fusion --depth 3 > gpurun_out/r05l_c5_fusion_errors.txt 2>&1 || { echo "stage errors rc=$?"; exit 1; }
timeout -k 10 150 python -u tools/gemm_bench.py --only flash > gpurun_out/r05l_flash.txt 2>&1 || { echo "gemm_bench rc=$?"; exit 1; }
bash tools/modeB_pmc.sh r05l_modeB || { echo "modeB pmc failed"; exit 1; }
echo done
