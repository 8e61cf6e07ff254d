#!/bin/bash
# tokres (proj / fc2 on the conv engine): its tests, the config-5 model tests, and a config-5 A/B.
set -o pipefail
OUT=gpurun_out/r06h; mkdir -p $OUT
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_flash_attn.py \
  tests/test_gpu_config5_b32.py tests/test_gpu_config5_full.py tests/test_gpu_transformer.py > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for r in 1 2; do for k in 1 0; do
  timeout -k 10 300 python3 bench.py --config 5 --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --knob tokres_conv=$k 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('tokres_conv=$k', d['value'], d['ms_per_step'])" || exit 1
done; done
