#!/bin/bash
# Interleaved mode-A A/B of existing knobs on the current tree: ROUNDS x variants, one bench process each.
# usage: gpurun -- bash tools/knob_sweep.sh TAG "k1=v1;k2=v2,k3=v3;..." [ROUNDS] [extra bench args]
set -o pipefail
TAG=${1:?tag}; VARS=${2:?variants}; ROUNDS=${3:-3}; shift 3; EXTRA="$*"
O=gpurun_out/$TAG; mkdir -p $O
IFS=';' read -ra VS <<< "$VARS"
for r in $(seq 1 $ROUNDS); do
  for v in "${VS[@]}"; do
    args=""
    IFS=',' read -ra KS <<< "$v"
    for k in "${KS[@]}"; do [ -n "$k" ] && [ "$k" != "default" ] && args="$args --knob $k"; done
    timeout -k 10 200 python bench.py --steps 40 --warmup 5 --no-extras --no-roofline --no-cpu-baseline $args $EXTRA 2>/dev/null \
      | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'], d['ms_per_step_median'])" >> $O/ab.txt || exit 1
  done
done
cat $O/ab.txt
