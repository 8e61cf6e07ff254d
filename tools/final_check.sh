#!/bin/bash
# Full GPU suite, the opt-in MFMA-linear path's parity tests, an interleaved A/B of it, and the recon
# kernels' per-launch time. usage: gpurun -- bash tools/final_check.sh TAG
set -o pipefail
TAG=${1:?tag}
ROOT=$(pwd); OUT=$ROOT/gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
DMF_LINEAR_MFMA=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_golden_full.py tests/test_gpu_dp.py -m gpu > $OUT/tests_mfma.log 2>&1; echo "mfma-linear tests rc=$?"; tail -1 $OUT/tests_mfma.log
bash tools/ab_env.sh 3 "DMF_LINEAR_MFMA=0" "DMF_LINEAR_MFMA=1" || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extras --no-roofline > $OUT/prof.log 2>&1 || { tail -5 $OUT/prof.log; exit 1; }
grep -E "recon|sgemm|k_gemm" $OUT/prof/run_kernel_stats.csv | cut -d, -f1,2,4 | cut -c1-160
