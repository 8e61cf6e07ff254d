#!/bin/bash
# rocprofv3 kernel stats of the encoder-forward replay + the conv microbench.
# usage: gpurun -- bash tools/prof_enc.sh TAG
set -o pipefail
TAG=${1:?tag}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 200 python tools/enc_fwd_prof.py --reps 20 > $OUT/enc.json 2> $OUT/enc.err || { tail -20 $OUT/enc.err; exit 1; }
cat $OUT/enc.json
timeout -k 10 200 python tools/enc_fwd_prof.py --reps 20 --serial > $OUT/enc_serial.json 2>> $OUT/enc.err || exit 1
cat $OUT/enc_serial.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $ROOT/tools/enc_fwd_prof.py --reps 20 --serial > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
cd $ROOT
timeout -k 10 300 python tools/conv_bench.py > $OUT/conv_bench.txt 2>&1 || { tail -20 $OUT/conv_bench.txt; exit 1; }
timeout -k 10 300 python tools/conv_bench.py --nostats > $OUT/conv_bench_nostats.txt 2>&1 || exit 1
cat $OUT/conv_bench.txt
