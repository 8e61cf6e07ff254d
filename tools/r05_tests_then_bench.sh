#!/bin/bash
# GPU: the whole -m gpu suite, then (only if pytest ended normally: 0 = passed, 1 = test failures)
# the token/fp8 GEMM microbench. Any other status (timeout, abort, fault) ends the script.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread tests \
  > gpurun_out/r05j_gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 150 python -u tools/gemm_bench.py --only fp8,flash > gpurun_out/r05j_gemm_bench.txt 2>&1
echo "gemm_bench rc=$?"
exit $rc
