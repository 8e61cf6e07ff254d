#!/bin/bash
# MFMA-busy / LDS counters of the bench step's kernels: two rocprofv3 --pmc passes (<= 8 SQ + 2 GRBM each),
# each its own run under a hard time limit (MI355X_MICROARCH.md "rocprofv3 PMC slots").
# usage: gpurun -- bash tools/pmc_mfma.sh TAG [bench args...]   (default bench args: mode A, --no-extras)
set -o pipefail
TAG=${1:?tag}; shift
ARGS=${*:---no-extras}
ROOT=$(pwd); OUT=$ROOT/gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq -o run -- python3 $ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-roofline $ARGS > $OUT/sq.log 2>&1 || { echo "pmc sq failed rc=$?"; tail -20 $OUT/sq.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $OUT/lds -o run -- python3 $ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-roofline $ARGS > $OUT/lds.log 2>&1 || { echo "pmc lds failed rc=$?"; tail -20 $OUT/lds.log; exit 1; }
cd $ROOT
python3 tools/pmc_mfma.py $OUT --by-kernel --json $OUT/pmc_mfma.json
