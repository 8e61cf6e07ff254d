#!/bin/bash
# ping-pong conv: correctness tests, then interleaved A/B timing against the current forms
set -o pipefail
TAG=${1:?tag}
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_conv_pp.py > $OUT/tests.log 2>&1 || { echo "tests failed rc=$?"; grep -E "PASSED|FAILED" $OUT/tests.log; tail -40 $OUT/tests.log; exit 1; }
grep -cE "PASSED" $OUT/tests.log
timeout -k 10 600 python tools/conv_bench.py --acc --tunes "7:0;7:2,8:0;7:2,8:1" --rounds 3 --only 1,2,3,7,8,10 > $OUT/ab.txt 2>&1 || { tail -20 $OUT/ab.txt; exit 1; }
cat $OUT/ab.txt
