#!/bin/bash
# SQ counters of the persistent (ps) vs ping-pong (pp) forward conv on chosen microbench shapes.
# usage: gpurun -- bash tools/pmc_pp.sh TAG "2,1"
set -o pipefail
TAG=${1:?tag}; ONLY=${2:-2}
ROOT=$(pwd); OUT=$ROOT/gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
ARGS="--tunes 7:0;7:2 --rounds 1 --reps 3 --acc --only $ONLY"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU --output-format csv -d $OUT/sq -o run -- python3 $ROOT/tools/conv_bench.py $ARGS > $OUT/sq.log 2>&1 || { tail -5 $OUT/sq.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $OUT/lds -o run -- python3 $ROOT/tools/conv_bench.py $ARGS > $OUT/lds.log 2>&1 || { tail -5 $OUT/lds.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 $ROOT/tools/conv_bench.py $ARGS > $OUT/kt.log 2>&1 || { tail -5 $OUT/kt.log; exit 1; }
cd $ROOT
python tools/pmc_summary.py $OUT/sq | grep -v "^   SQ_WAVES"
python tools/pmc_summary.py $OUT/lds
f=$(find $OUT/kt -name '*kernel_stats.csv' | head -1); grep -E "conv_fwd" "$f" | cut -c1-160
