#!/bin/bash
# One gpurun session: GPU parity tests, a short bench, a rocprofv3 kernel-stats pass.
# usage: gpurun -- bash tools/gpu_session.sh [tag] [what]   (what: all|tests|bench|prof)
set -o pipefail
TAG=${1:-run}
WHAT=${2:-all}
OUT=gpurun_out/$TAG
mkdir -p $OUT
ROOT=$(pwd)
if [ "$WHAT" = all ] || [ "$WHAT" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rf --durations=25 --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed rc=$?"; tail -40 $OUT/tests.log; exit 1; }
  tail -3 $OUT/tests.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed rc=$?"; tail -30 $OUT/smoke.log; exit 1; }
  tail -2 $OUT/smoke.log
fi
if [ "$WHAT" = all ] || [ "$WHAT" = bench ]; then
  DMF_CONV_DUMP=$OUT/conv.jsonl timeout -k 10 600 python bench.py ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed rc=$?"; tail -30 $OUT/bench.err; exit 1; }
  cat $OUT/bench.json
fi
if [ "$WHAT" = all ] || [ "$WHAT" = prof ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/prof -o run -- python3 $ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS} > $ROOT/$OUT/prof.log 2>&1 || { echo "prof failed rc=$?"; tail -30 $ROOT/$OUT/prof.log; exit 1; }
  cd $ROOT
  f=$(find $OUT/prof -name '*kernel_stats.csv' | head -1)
  echo "stats: $f"
  head -25 "$f" | cut -c1-200
fi
