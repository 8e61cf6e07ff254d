#!/bin/bash
set -o pipefail
OUT=gpurun_out/r03e; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_conv_stem.py tests/test_gpu_shortcut_handoff.py > $OUT/stem_tests.log 2>&1 || { grep -E "PASS|FAIL|Error|assert" $OUT/stem_tests.log | tail -30; exit 1; }
tail -1 $OUT/stem_tests.log
timeout -k 10 300 python tools/conv_bench.py --acc --tunes "10:1;10:0" --rounds 3 --only 12,13 > $OUT/stem_ab.txt 2>&1 || { tail -20 $OUT/stem_ab.txt; exit 1; }
cat $OUT/stem_ab.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { grep -E "FAIL|Error" $OUT/tests.log | tail -20; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['encoder_forward']['ms'], d['mode_b']['value'], d['config2']['value'])"
