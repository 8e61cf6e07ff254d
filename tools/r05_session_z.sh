#!/bin/bash
# r05z: fc1 + GELU + dropout on the conv engine: tests, microbench, config-5 bench A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  tests/test_gpu_flash_attn.py tests/test_gpu_transformer.py tests/test_gpu_config5_b32.py > gpurun_out/r05z_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r05z_tests.log; exit 1; }
tail -2 gpurun_out/r05z_tests.log
timeout -k 10 150 python -u tools/gemm_bench.py --only fc1 > gpurun_out/r05z_gemm.txt 2>&1 || exit 1
grep -v "Warn\|amdgpu" gpurun_out/r05z_gemm.txt
for i in 1 2; do
  for v in 1 0; do
    timeout -k 10 300 python bench.py --config 5 --size 384 --no-extras --no-cpu-baseline --no-roofline --steps 20 --warmup 3 --knob fc1_drop_conv=$v > gpurun_out/r05z_c5_$v.$i.json 2> gpurun_out/r05z_c5_$v.$i.err || { echo "bench rc=$?"; tail -5 gpurun_out/r05z_c5_$v.$i.err; exit 1; }
    echo "fc1_drop_conv=$v round $i: $(cut -c1-140 gpurun_out/r05z_c5_$v.$i.json)"
  done
done
