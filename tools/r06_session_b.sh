set -o pipefail
mkdir -p gpurun_out/r06b
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_eval_fold.py tests/test_gpu_configs.py tests/test_gpu_two_pass_bn.py tests/test_gpu_conv_stem.py > gpurun_out/r06b/tests.log 2>&1 || { tail -40 gpurun_out/r06b/tests.log; exit 1; }
tail -3 gpurun_out/r06b/tests.log
for k in 0 1; do timeout -k 10 200 python3 bench.py --config 2 --steps 50 --warmup 10 --knob eval_bn_fold=$k 2>/dev/null | tail -1 | cut -c1-330; done
