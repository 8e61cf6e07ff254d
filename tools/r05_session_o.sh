#!/bin/bash
# r05o: packed-fp32 GELU: exactness tests, the BN-apply / fc1 microbenches, then the GELU-bearing kernel tests.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  tests/test_gpu_gelu_packed.py tests/test_gpu_kernels.py tests/test_gpu_transformer.py tests/test_gpu_vit.py > gpurun_out/r05o_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r05o_tests.log; exit 1; }
tail -2 gpurun_out/r05o_tests.log
timeout -k 10 200 python -u tools/apply_bench.py > gpurun_out/r05o_apply.txt 2>&1 || { echo "apply rc=$?"; exit 1; }
grep -v Warn gpurun_out/r05o_apply.txt | tail -13
timeout -k 10 150 python -u tools/gemm_bench.py --only fc1 > gpurun_out/r05o_fc1.txt 2>&1 || { echo "gemm rc=$?"; exit 1; }
grep -v Warn gpurun_out/r05o_fc1.txt | tail -3
