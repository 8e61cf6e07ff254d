#!/bin/bash
# conv parity tests + interleaved A/B of dmf_conv_tune variants on the GPU box
# usage: bash tools/conv_ab.sh TAG "TUNES" [ONLY]
set -o pipefail
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q -k conv --timeout 180 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "conv tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 500 python tools/conv_bench.py --from profiles/r01g_conv_launches.jsonl --tunes "$2" ${3:+--only $3} > $OUT/ab.txt 2>&1 || { tail -20 $OUT/ab.txt; exit 1; }
cat $OUT/ab.txt
