#!/bin/bash
# Mode-B kernel trace (timeline + stats) and the torch-op census of one eager mode-B step.
# usage: gpurun -- bash tools/prof_modeB.sh TAG
set -o pipefail
TAG=${1:?tag}
ROOT=$(pwd); OUT=$ROOT/gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 300 python3 tools/trace_ops.py --mode B --batch 32 > $OUT/ops.txt 2>&1 || { tail -20 $OUT/ops.txt; exit 1; }
head -40 $OUT/ops.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/profB -o run -- python3 $ROOT/bench.py --mode B --steps 6 --warmup 2 --no-cpu-baseline --no-extras --no-roofline > $OUT/profB.log 2>&1 || { tail -20 $OUT/profB.log; exit 1; }
tail -c 300 $OUT/profB.log
cd $ROOT
for f in $(find $OUT -name '*kernel_trace.csv'); do gzip $f; done
