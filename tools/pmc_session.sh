#!/bin/bash
# HBM traffic of the bench step's kernels: one rocprofv3 --pmc pass per counter
# (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).
# usage: gpurun -- bash tools/pmc_session.sh [tag]
set -o pipefail
TAG=${1:-pmc}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d $OUT/$C -o run -- python3 $ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-roofline ${BENCH_ARGS} > $OUT/$C.log 2>&1 || { echo "pmc $C failed rc=$?"; tail -20 $OUT/$C.log; exit 1; }
done
ls -R $OUT | head -20
