#!/bin/bash
# Weight re-layout A/B (mode B re-prepares every trainable conv weight each step): rocprofv3 kernel stats of a
# short mode-B bench per library variant, then interleaved whole-step A/B. usage: bash tools/wprep_ab.sh A B
set -o pipefail
ROOT=$(pwd); OUT=$ROOT/gpurun_out/wprep; mkdir -p $OUT
for n in "$@"; do
  (cd /tmp && export TMPDIR=/tmp DMF_HIP_LIB=$ROOT/ab/$n.so && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$n -o run -- python3 $ROOT/bench.py --mode B --steps 6 --warmup 2 --no-cpu-baseline --no-extras --no-roofline > $OUT/$n.log 2>&1) || { echo "prof $n failed"; tail -20 $OUT/$n.log; exit 1; }
  grep -h "k_weight_prep_multi\|k_adamw" $(find $OUT/$n -name '*kernel_stats.csv') | cut -c1-160
  find $OUT/$n -name '*kernel_trace.csv' -delete
done
AB_ARGS="--mode B --no-roofline" timeout -k 10 900 bash tools/ab_bench.sh 2 "$@"
