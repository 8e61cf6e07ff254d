set -o pipefail
mkdir -p gpurun_out/r03c
DMF_REPORT_DIR=gpurun_out/r03c timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_gpu_fit.py tests/test_gpu_amp.py tests/test_gpu_config5_full.py > gpurun_out/r03c/tests.log 2>&1 || { echo "tests failed rc=$?"; tail -60 gpurun_out/r03c/tests.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/r03c/tests.log | tail -12
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /root/repo/gpurun_out/r03c/prof -o run -- python3 /root/repo/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras > /root/repo/gpurun_out/r03c/prof.log 2>&1 || { echo "prof failed"; tail -20 /root/repo/gpurun_out/r03c/prof.log; exit 1; }
f=$(find /root/repo/gpurun_out/r03c/prof -name '*kernel_stats.csv' | head -1)
grep -i "recon" "$f" | cut -c1-200
