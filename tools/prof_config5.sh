#!/bin/bash
# Config-5 kernel stats of the bench step (rocprofv3 kernel trace + stats). usage: gpurun -- bash tools/prof_config5.sh TAG
set -o pipefail
TAG=${1:?tag}
ROOT=$(pwd); OUT=$ROOT/gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $ROOT/bench.py --config 5 --size 384 --steps 6 --warmup 2 --no-cpu-baseline --no-extras --no-roofline > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
tail -c 300 $OUT/prof.log
