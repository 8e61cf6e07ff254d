#!/bin/bash
# encoder-forward (north star) interleaved A/B over dmf_conv_tune settings, one process
# usage: gpurun -- bash tools/enc_ab.sh TAG "7:0;7:1" [rounds]
set -o pipefail
TAG=${1:?tag}; TUNES=${2:?tunes}; R=${3:-4}
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python tools/enc_fwd_ab.py --tunes "$TUNES" --rounds $R > $OUT/enc_ab.txt 2>&1 || { tail -20 $OUT/enc_ab.txt; exit 1; }
cat $OUT/enc_ab.txt
