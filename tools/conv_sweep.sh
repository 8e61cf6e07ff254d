#!/bin/bash
# conv microbench variants on the GPU box: default / no persistent / no stats
set -o pipefail
OUT=gpurun_out/${1:-cs}
mkdir -p $OUT
SRC=${2:-profiles/r01b_conv_launches.jsonl}
timeout -k 10 200 python tools/conv_bench.py --from $SRC > $OUT/default.txt 2>&1 || { tail -20 $OUT/default.txt; exit 1; }
DMF_CONV_NOPERS=1 timeout -k 10 200 python tools/conv_bench.py --from $SRC > $OUT/nopers.txt 2>&1 || exit 1
timeout -k 10 200 python tools/conv_bench.py --from $SRC --nostats > $OUT/nostats.txt 2>&1 || exit 1
paste $OUT/default.txt $OUT/nopers.txt $OUT/nostats.txt | awk -F'\t' '{print $1 " | " substr($2,index($2,"us")-9) " | " substr($3,index($3,"us")-9)}'
