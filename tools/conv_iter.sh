#!/bin/bash
# Conv iteration on the GPU box: conv parity tests, per-shape microbench,
# optional SQ counter pass on one shape.  usage: bash tools/conv_iter.sh TAG [ONLY] [PMC]
set -o pipefail
TAG=${1:?tag}
ONLY=${2:-}
OUT=gpurun_out/$TAG
mkdir -p $OUT
ROOT=$(pwd)
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k conv --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "conv tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python tools/conv_bench.py --from profiles/r01g_conv_launches.jsonl > $OUT/cb.txt 2>&1 || { tail -20 $OUT/cb.txt; exit 1; }
cat $OUT/cb.txt
if [ -n "$3" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -s KILL 120 rocprofv3 --pmc $3 --output-format csv -d $ROOT/$OUT/pmc -o run -- python3 $ROOT/tools/conv_bench.py --from $ROOT/profiles/r01g_conv_launches.jsonl --only $ONLY --reps 5 > $ROOT/$OUT/pmc.log 2>&1 || { echo "pmc failed"; tail -20 $ROOT/$OUT/pmc.log; exit 1; }
  cd $ROOT
  python tools/pmc_summary.py $OUT/pmc
fi
