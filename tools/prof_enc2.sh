#!/bin/bash
set -o pipefail
TAG=$1
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 200 python tools/enc_fwd_prof.py --reps 20 > $OUT/enc.json 2> $OUT/enc.err || { tail -20 $OUT/enc.err; exit 1; }
timeout -k 10 200 python tools/enc_fwd_prof.py --reps 20 --serial > $OUT/enc_serial.json 2>> $OUT/enc.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $ROOT/tools/enc_fwd_prof.py --reps 10 --serial > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
