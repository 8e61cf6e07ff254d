#!/bin/bash
# conv-forward A/Bs in one GPU call (training-forward mode: BN statistics into the arena)
# usage: gpurun -- bash tools/r03_ab.sh TAG "<tunes>" [only]
set -o pipefail
TAG=${1:?tag}; TUNES=${2:?tunes}; ONLY=${3:-}
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python tools/conv_bench.py --acc --tunes "$TUNES" --rounds 3 ${ONLY:+--only $ONLY} > $OUT/ab.txt 2>&1 || { tail -20 $OUT/ab.txt; exit 1; }
cat $OUT/ab.txt
