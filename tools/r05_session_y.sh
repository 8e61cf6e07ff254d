#!/bin/bash
# r05y: Philox (seed, offset) hoisted out of the dropout loops: mask tests, the token / attention benches.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  tests/test_gpu_flash_attn.py tests/test_gpu_transformer.py tests/test_gpu_determinism.py tests/test_gpu_kernels.py tests/test_gpu_predict_oracle.py > gpurun_out/r05y_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r05y_tests.log; exit 1; }
tail -2 gpurun_out/r05y_tests.log
timeout -k 10 150 python -u tools/gemm_bench.py --only flash,fc1,softmax > gpurun_out/r05y_gemm.txt 2>&1 || exit 1
grep -v "Warn\|amdgpu" gpurun_out/r05y_gemm.txt
