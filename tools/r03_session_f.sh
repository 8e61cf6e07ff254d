#!/bin/bash
set -o pipefail
OUT=gpurun_out/r03f; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv_pp.py tests/test_gpu_golden_full.py tests/test_gpu_conv_stem.py > $OUT/tests.log 2>&1 || { grep -E "FAIL|Error|assert" $OUT/tests.log | tail -30; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 600 python tools/conv_bench.py --acc --tunes "11:1;11:0" --rounds 3 > $OUT/ab.txt 2>&1 || { tail -20 $OUT/ab.txt; exit 1; }
cat $OUT/ab.txt
timeout -k 10 300 python tools/enc_fwd_ab.py --tunes "11:1;11:0" --rounds 4 > $OUT/enc_ab.txt 2>&1 || { tail -20 $OUT/enc_ab.txt; exit 1; }
tail -5 $OUT/enc_ab.txt
