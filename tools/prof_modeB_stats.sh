#!/bin/bash
# Mode-B kernel trace + stats of the bench step (no op census): usage: gpurun -- bash tools/prof_modeB_stats.sh TAG
set -o pipefail
TAG=${1:?tag}
ROOT=$(pwd); OUT=$ROOT/gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/profB -o run -- python3 $ROOT/bench.py --mode B --steps 6 --warmup 2 --no-cpu-baseline --no-extras --no-roofline > $OUT/profB.log 2>&1 || { tail -20 $OUT/profB.log; exit 1; }
tail -c 300 $OUT/profB.log
cd $ROOT
python3 tools/timeline.py $(find $OUT -name '*kernel_trace.csv' | head -1) --last 1 --top 40 > $OUT/timeline.txt 2>&1
for f in $(find $OUT -name '*kernel_trace.csv'); do gzip $f; done
head -50 $OUT/timeline.txt
