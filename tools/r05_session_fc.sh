#!/bin/bash
# r05fc: BN backward apply with the first row group loaded before its finalize prologue: parity
# tests, then mode B and mode A bench lines (against r05f3: mode B 1047.7, mode A 3408.6 vol/s).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  tests/test_gpu_bn_apply_rows.py tests/test_gpu_two_pass_bn.py > gpurun_out/r05fc_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r05fc_tests.log; exit 1; }
tail -2 gpurun_out/r05fc_tests.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --mode B --no-extras --no-cpu-baseline --no-roofline --steps 25 --warmup 3 > gpurun_out/r05fc_b.$i.json 2> gpurun_out/r05fc_b.$i.err || { echo "bench rc=$?"; tail -5 gpurun_out/r05fc_b.$i.err; exit 1; }
  echo "mode B run $i: $(cut -c1-140 gpurun_out/r05fc_b.$i.json)"
  timeout -k 10 300 python bench.py --no-extras --no-cpu-baseline --no-roofline --steps 50 --warmup 10 > gpurun_out/r05fc_a.$i.json 2> gpurun_out/r05fc_a.$i.err || { echo "bench rc=$?"; tail -5 gpurun_out/r05fc_a.$i.err; exit 1; }
  echo "mode A run $i: $(cut -c1-140 gpurun_out/r05fc_a.$i.json)"
done
