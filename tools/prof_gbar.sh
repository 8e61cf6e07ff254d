#!/bin/bash
# per-kernel split of the serial encoder forward with the grid-barrier BN apply on and off
set -o pipefail
TAG=$1
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for v in 1 0; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof$v -o run -- python3 $ROOT/tools/enc_fwd_prof.py --reps 5 --serial --knob grid_barrier_bn=$v > $OUT/prof$v.log 2>&1 || { tail -20 $OUT/prof$v.log; exit 1; }
done
