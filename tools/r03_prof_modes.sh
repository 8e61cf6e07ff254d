#!/bin/bash
# rocprofv3 kernel traces of mode A alone, mode B alone (bench.py --no-extras) and the
# two-stream encoder forward. usage: gpurun -- bash tools/r03_prof_modes.sh TAG
set -o pipefail
TAG=${1:?tag}
ROOT=$(pwd); OUT=$ROOT/gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/profA -o run -- python3 $ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras --no-roofline > $OUT/profA.log 2>&1 || { tail -20 $OUT/profA.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/profB -o run -- python3 $ROOT/bench.py --mode B --steps 10 --warmup 2 --no-cpu-baseline --no-extras --no-roofline > $OUT/profB.log 2>&1 || { tail -20 $OUT/profB.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/profE -o run -- python3 $ROOT/tools/enc_fwd_prof.py --reps 10 > $OUT/profE.log 2>&1 || { tail -20 $OUT/profE.log; exit 1; }
tail -1 $OUT/profA.log | cut -c1-300; tail -1 $OUT/profB.log | cut -c1-300
