#!/bin/bash
# Kernel trace of a short mode-A bench and the copy census of its last step: gpurun -- bash tools/copy_prof.sh TAG [bench args]
set -o pipefail
TAG=${1:?tag}; shift
ROOT=$(pwd); OUT=$ROOT/gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- python3 $ROOT/bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-extras --no-roofline "$@" > $OUT/prof.log 2>&1 || { echo "prof failed"; tail -20 $OUT/prof.log; exit 1; }
cd $ROOT
python3 tools/copy_census.py $(find $OUT -name '*kernel_trace.csv' | head -1) > $OUT/census.txt 2>&1
for f in $(find $OUT -name '*kernel_trace.csv'); do gzip $f; done
cat $OUT/census.txt
