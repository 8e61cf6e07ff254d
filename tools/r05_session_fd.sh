#!/bin/bash
# r05fd: GroupNorm applies on 8-channel vectors: GN tests, mode-A kernel stats, mode A / B bench lines.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  tests/test_gpu_kernels.py -k "gn_mix" > gpurun_out/r05fd_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r05fd_tests.log; exit 1; }
tail -2 gpurun_out/r05fd_tests.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r05fd_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-extras --no-cpu-baseline --no-roofline --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/r05fd_prof.json 2> $GRAFT_REPO_ROOT/gpurun_out/r05fd_prof.err || { echo "prof rc=$?"; tail -5 $GRAFT_REPO_ROOT/gpurun_out/r05fd_prof.err; exit 1; }
cd $GRAFT_REPO_ROOT
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-extras --no-cpu-baseline --no-roofline --steps 50 --warmup 10 > gpurun_out/r05fd_a.$i.json 2> gpurun_out/r05fd_a.$i.err || { echo "bench rc=$?"; tail -5 gpurun_out/r05fd_a.$i.err; exit 1; }
  echo "mode A run $i: $(cut -c1-140 gpurun_out/r05fd_a.$i.json)"
done
