#!/bin/bash
# tests + the bench lines of one round: config 3 mode A (headline), config 3 mode B, config 5 mode A/B
# usage: bash tools/bench_matrix.sh TAG [skip-tests]
set -o pipefail
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ -z "$2" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
  tail -1 $OUT/tests.log
fi
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $OUT/c3A.json 2> $OUT/c3A.err || { echo "c3A failed"; tail -20 $OUT/c3A.err; exit 1; }
cat $OUT/c3A.json
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --mode B --no-cpu-baseline > $OUT/c3B.json 2> $OUT/c3B.err || { echo "c3B failed"; tail -20 $OUT/c3B.err; exit 1; }
cat $OUT/c3B.json
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --config 5 --no-cpu-baseline > $OUT/c5A.json 2> $OUT/c5A.err || { echo "c5A failed"; tail -20 $OUT/c5A.err; exit 1; }
cat $OUT/c5A.json
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --config 5 --mode B --no-cpu-baseline --no-roofline > $OUT/c5B.json 2> $OUT/c5B.err || { echo "c5B failed"; tail -20 $OUT/c5B.err; exit 1; }
cat $OUT/c5B.json
