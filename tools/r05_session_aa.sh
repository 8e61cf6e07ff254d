#!/bin/bash
# r05aa: rows in flight in the BN-backward apply (knob bwd_apply_rows), mode-B A/B + the backward tests.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_modeb_wgrad.py > gpurun_out/r05aa_tests.log 2>&1 || { echo "tests rc=$?"; tail -20 gpurun_out/r05aa_tests.log; exit 1; }
tail -1 gpurun_out/r05aa_tests.log
for i in 1 2; do
  for v in 1 2 4; do
    timeout -k 10 200 python bench.py --mode B --no-extras --no-cpu-baseline --no-roofline --steps 25 --warmup 5 --knob bwd_apply_rows=$v > gpurun_out/r05aa_modeB_$v.$i.json 2> gpurun_out/r05aa_modeB_$v.$i.err || { echo "bench rc=$?"; tail -5 gpurun_out/r05aa_modeB_$v.$i.err; exit 1; }
    echo "bwd_apply_rows=$v round $i: $(cut -c1-140 gpurun_out/r05aa_modeB_$v.$i.json)"
  done
done
