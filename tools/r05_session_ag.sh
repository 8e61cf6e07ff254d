#!/bin/bash
# r05ag: the fusion's fp32 GEMMs on fp32-MFMA tiles: tests, per-shape timing, mode-A A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_sgemm.py tests/test_gpu_parity.py tests/test_gpu_determinism.py tests/test_gpu_dp.py > gpurun_out/r05ag_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r05ag_tests.log; exit 1; }
tail -1 gpurun_out/r05ag_tests.log
timeout -k 10 200 python -u tools/sgemm_shapes.py > gpurun_out/r05ag_sgemm_shapes.txt 2>&1 || exit 1
grep -v "Warn\|amdgpu\|warn" gpurun_out/r05ag_sgemm_shapes.txt | tail -16
for i in 1 2 3; do
  for v in 1 0; do
    timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline --no-roofline --steps 50 --warmup 10 --knob sgemm_mfma=$v > gpurun_out/r05ag_modeA_$v.$i.json 2> gpurun_out/r05ag_modeA_$v.$i.err || { echo "bench rc=$?"; tail -5 gpurun_out/r05ag_modeA_$v.$i.err; exit 1; }
    echo "sgemm_mfma=$v round $i: $(cut -c1-140 gpurun_out/r05ag_modeA_$v.$i.json)"
  done
done
