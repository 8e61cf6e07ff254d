#!/bin/bash
# Selected -m gpu tests, then a kernel-stats profile of the encoder-forward replay with the
# kernels matching a pattern. usage: gpurun -- bash tools/quick_enc.sh TAG "<pytest -k expr>" "<grep pattern>"
set -o pipefail
TAG=${1:?tag}; KSEL=${2:-}; PAT=${3:-.}
ROOT=$(pwd); OUT=$ROOT/gpurun_out/$TAG; mkdir -p $OUT
if [ -n "$KSEL" ]; then
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu -k "$KSEL" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
  tail -1 $OUT/tests.log
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $ROOT/tools/enc_fwd_prof.py --reps 10 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
grep -v rocprofv3 $OUT/prof.log | tail -2
grep -E "$PAT" $OUT/prof/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-200
