#!/bin/bash
# One bounded GPU call: selected -m gpu tests, then (optionally) a rocprofv3 kernel-stats pass of a
# short bench and the kernels matching a pattern.
# usage: gpurun -- bash tools/gpu_quick.sh TAG "<pytest selection>" ["<kernel grep pattern>"] ["<bench args>"]
set -o pipefail
TAG=${1:?tag}; SEL=${2:-}; PAT=${3:-}; BARGS=${4:---no-extras}
ROOT=$(pwd); OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
if [ -n "$SEL" ]; then
  DMF_REPORT_DIR=$OUT timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread $SEL > $OUT/tests.log 2>&1 || { echo "tests failed rc=$?"; grep -E "PASSED|FAILED|Error" $OUT/tests.log | tail -20; tail -40 $OUT/tests.log; exit 1; }
  grep -cE "PASSED" $OUT/tests.log; tail -1 $OUT/tests.log
fi
if [ -n "$PAT" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline $BARGS > $OUT/prof.log 2>&1 || { echo "prof failed rc=$?"; tail -20 $OUT/prof.log; exit 1; }
  f=$(find $OUT/prof -name '*kernel_stats.csv' | head -1)
  head -1 "$f" | cut -c1-200
  grep -iE "$PAT" "$f" | cut -c1-220 || true
  tail -1 $OUT/prof.log | cut -c1-600
fi
