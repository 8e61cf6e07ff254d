#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_se_mlp.py tests/test_gpu_parity.py > gpurun_out/r05ai_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r05ai_tests.log; exit 1; }
tail -1 gpurun_out/r05ai_tests.log
timeout -k 10 120 python -u tools/se_bench.py > gpurun_out/r05ai_se_bench.txt 2>&1 || exit 1
grep -v "Warn\|amdgpu" gpurun_out/r05ai_se_bench.txt
for i in 1 2; do
  for v in 1 0; do
    timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline --no-roofline --steps 50 --warmup 10 --knob se_one_launch=$v > gpurun_out/r05ai_modeA_$v.$i.json 2> gpurun_out/r05ai_modeA_$v.$i.err || { echo "bench rc=$?"; tail -5 gpurun_out/r05ai_modeA_$v.$i.err; exit 1; }
    echo "se_one_launch=$v round $i: $(cut -c1-140 gpurun_out/r05ai_modeA_$v.$i.json)"
  done
done
