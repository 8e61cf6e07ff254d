#!/bin/bash
# HBM traffic per weight-gradient launch (MFMA wgrad kernel + its split reduce) of the mode-B bench step:
# the two rocprofv3 --pmc passes of tools/pmc_session.sh on `bench.py --mode B`, summarised per pair.
# usage: gpurun -- bash tools/modeB_pmc.sh TAG
set -o pipefail
TAG=${1:?tag}
BENCH_ARGS="--no-extras --mode B" bash tools/pmc_session.sh ${TAG}_pmc > /dev/null || exit 1
python tools/pmc_traffic.py gpurun_out/${TAG}_pmc --match 'k_conv_wgrad(_dma|_tr)?[<(]|k_wgrad_reduce' \
  --count 'k_conv_wgrad(_dma|_tr)?[<(]' --json gpurun_out/${TAG}_pmc_traffic_wgrad.json
