#!/bin/bash
# L2 behaviour of conv microbench shapes: hit/miss, fetched and written bytes (separate passes).
# usage: gpurun -- bash tools/pmc_l2.sh TAG "1,3"
set -o pipefail
TAG=${1:?tag}; ONLY=${2:-1}
ROOT=$(pwd); OUT=$ROOT/gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for P in "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE" "TCP_TCC_READ_REQ_sum TCC_EA0_RDREQ_sum"; do
  N=$(echo $P | tr ' ' '_')
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/$N -o run -- python3 $ROOT/tools/conv_bench.py --only $ONLY --reps 3 > $OUT/$N.log 2>&1 || { echo "pass $P failed"; tail -5 $OUT/$N.log; exit 1; }
done
cd $ROOT
for d in $OUT/*/; do python tools/pmc_summary.py $d | grep -A4 "k_conv_fwd"; done
