#!/bin/bash
# r05fb: BN apply (first row group loaded before the finalize prologue) with 1 / 2 / 4 rows of loads in flight per thread: parity test, microbench, mode-A A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  tests/test_gpu_bn_apply_rows.py tests/test_gpu_gelu_packed.py > gpurun_out/r05fb_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r05fb_tests.log; exit 1; }
tail -2 gpurun_out/r05fb_tests.log
for u in 1 2 4; do
  timeout -k 10 120 python -u tools/apply_bench.py --rows $u > gpurun_out/r05fb_apply_$u.txt 2>&1 || exit 1
  echo "rows=$u"; grep -v "Warn\|amdgpu" gpurun_out/r05fb_apply_$u.txt
done
for i in 1 2; do
  for v in 1 4 2; do
    timeout -k 10 300 python bench.py --no-extras --no-cpu-baseline --no-roofline --steps 50 --warmup 10 --knob fwd_apply_rows=$v > gpurun_out/r05fb_a_$v.$i.json 2> gpurun_out/r05fb_a_$v.$i.err || { echo "bench rc=$?"; tail -5 gpurun_out/r05fb_a_$v.$i.err; exit 1; }
    echo "fwd_apply_rows=$v round $i: $(cut -c1-140 gpurun_out/r05fb_a_$v.$i.json)"
  done
done
