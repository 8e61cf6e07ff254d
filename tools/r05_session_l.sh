#!/bin/bash
# r05l: two-pass fold tests + encoder-forward A/B, config-5 fusion-stage errors, the flash-attention bench
# after the Philox change, the mode-B PMC traffic passes. Each GPU step under its own limit; a non-zero
# status ends the script.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  tests/test_gpu_two_pass_bn.py tests/test_gpu_flash_attn.py > gpurun_out/r05l_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r05l_tests.log; exit 1; }
tail -2 gpurun_out/r05l_tests.log
timeout -k 10 300 python -u tools/enc_fwd_ab.py --tunes "two_pass_fold=1;two_pass_fold=0" --rounds 5 > gpurun_out/r05l_fold_ab.txt 2>&1 || { echo "ab rc=$?"; exit 1; }
tail -4 gpurun_out/r05l_fold_ab.txt
timeout -k 10 400 python -u tools/config5_stage_errors.py --fusion --depth 3 > gpurun_out/r05l_c5_fusion_errors.txt 2>&1 || { echo "stage errors rc=$?"; exit 1; }
timeout -k 10 150 python -u tools/gemm_bench.py --only flash > gpurun_out/r05l_flash.txt 2>&1 || { echo "gemm_bench rc=$?"; exit 1; }
bash tools/modeB_pmc.sh r05l_modeB || { echo "modeB pmc failed"; exit 1; }
echo done
