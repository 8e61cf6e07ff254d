#!/bin/bash
# Kernel traces (start/end timestamps, no counters) of the encoder forward replay and of a short
# mode-A bench, for tools/timeline.py. usage: gpurun -- bash tools/trace_session.sh TAG
set -o pipefail
TAG=${1:?tag}
ROOT=$(pwd); OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/enc -o enc -- python3 $ROOT/tools/enc_fwd_prof.py --reps 10 > $OUT/enc.log 2>&1 || { echo "enc trace failed rc=$?"; tail -20 $OUT/enc.log; exit 1; }
tail -2 $OUT/enc.log
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/step -o step -- python3 $ROOT/bench.py --steps 6 --warmup 2 --no-extras --no-cpu-baseline --no-roofline > $OUT/step.log 2>&1 || { echo "step trace failed rc=$?"; tail -20 $OUT/step.log; exit 1; }
tail -c 400 $OUT/step.log
cd $ROOT
for f in $(find $OUT -name '*kernel_trace.csv'); do gzip -k $f; ls -la $f.gz; done
