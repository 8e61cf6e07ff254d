#!/bin/bash
# Checkpoint of a tree: the whole GPU suite, smoke(), then the default bench line.
# usage: gpurun --timeout 1200 -- bash tools/full_check.sh TAG [--no-bench]
set -o pipefail
TAG=${1:?tag}
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
[ "$2" = "--no-bench" ] && exit 0
timeout -k 10 500 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.json | cut -c1-600
