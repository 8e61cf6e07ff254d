#!/bin/bash
# Round-6 session A: the changed tests, the two-stream overlap with and without the profiler,
# MFMA/LDS counters for mode A and mode B, and the default bench line.
# usage: gpurun --timeout 1200 -- bash tools/r06_session_a.sh
set -o pipefail
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r06a; mkdir -p $OUT
export TMPDIR=/tmp
step() { echo "== $(date +%T) $*"; }
step tests
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_flash_attn.py tests/test_gpu_dp.py "tests/test_gpu_transformer.py::test_hybrid_encoder_under_16_mixed" \
  > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
step "encoder forward, two streams vs one, no profiler"
timeout -k 10 240 python3 tools/enc_fwd_ab.py --tunes "parallel_encoders=1;parallel_encoders=0" --rounds 3 > $OUT/enc_ab_noprof.txt 2>&1 || { tail -20 $OUT/enc_ab_noprof.txt; exit 1; }
cat $OUT/enc_ab_noprof.txt | grep variant
step "the same under rocprofv3 --kernel-trace"
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python3 $ROOT/tools/enc_fwd_ab.py --tunes "parallel_encoders=1;parallel_encoders=0" --rounds 3 > $OUT/enc_ab_prof.txt 2>&1 ) || { tail -20 $OUT/enc_ab_prof.txt; exit 1; }
grep variant $OUT/enc_ab_prof.txt
step "mfma counters mode A"
bash tools/pmc_mfma.sh r06a_pmcA --no-extras > $OUT/pmcA.txt 2>&1 || { tail -20 $OUT/pmcA.txt; exit 1; }
head -12 $OUT/pmcA.txt
step "mfma counters mode B"
bash tools/pmc_mfma.sh r06a_pmcB --mode B --no-extras > $OUT/pmcB.txt 2>&1 || { tail -20 $OUT/pmcB.txt; exit 1; }
head -8 $OUT/pmcB.txt
step bench
timeout -k 10 400 python3 bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-400
step done
