#!/bin/bash
# SQ counters of the conv microbench shapes (one pass, <= 8 SQ counters).
# usage: gpurun -- bash tools/pmc_conv.sh TAG "1,3,7"
set -o pipefail
TAG=${1:?tag}; ONLY=${2:-1,3,7}
ROOT=$(pwd); OUT=$ROOT/gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU --output-format csv -d $OUT/sq -o run -- python3 $ROOT/tools/conv_bench.py --only $ONLY --reps 3 > $OUT/sq.log 2>&1 || { tail -5 $OUT/sq.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $OUT/lds -o run -- python3 $ROOT/tools/conv_bench.py --only $ONLY --reps 3 > $OUT/lds.log 2>&1 || { tail -5 $OUT/lds.log; exit 1; }
cd $ROOT
python tools/pmc_summary.py $OUT/sq | grep -v "^   SQ_WAVES" 
python tools/pmc_summary.py $OUT/lds
