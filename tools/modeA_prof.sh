#!/bin/bash
# Mode-A-only evidence for the bench line's dominant-kernel roofline: rocprofv3 kernel stats of the
# default bench without the sub-lines (so the conv-forward family average is mode A's), and the two
# PMC traffic passes of the same run. usage: gpurun -- bash tools/modeA_prof.sh TAG
set -o pipefail
TAG=${1:?tag}
ROOT=$(pwd); OUT=$ROOT/gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras > $OUT/prof.log 2>&1 || { echo "prof failed"; tail -20 $OUT/prof.log; exit 1; }
tail -1 $OUT/prof.log | cut -c1-300
cd $ROOT
BENCH_ARGS=--no-extras bash tools/pmc_session.sh ${TAG}_pmc > /dev/null || exit 1
python tools/pmc_traffic.py gpurun_out/${TAG}_pmc --json gpurun_out/$TAG/pmc_traffic.json
