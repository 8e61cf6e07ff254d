#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r03d
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "recon" > gpurun_out/r03d/recon_tests.log 2>&1 || { tail -30 gpurun_out/r03d/recon_tests.log; exit 1; }
tail -1 gpurun_out/r03d/recon_tests.log
bash tools/r03_prof_modes.sh r03d
