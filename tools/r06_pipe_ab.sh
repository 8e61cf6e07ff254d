#!/bin/bash
# Mode-A pipelined vs sequential steps under stream / queue variants (round 6 A/B).
set -e
O=gpurun_out/r06j; mkdir -p $O
B="python bench.py --steps 40 --warmup 5 --no-extras --no-roofline --no-cpu-baseline"
for r in 1 2; do
  timeout -k 10 200 $B > $O/pip_$r.json 2>> $O/err.txt
  timeout -k 10 200 $B --no-pipeline > $O/seq_$r.json 2>> $O/err.txt
  timeout -k 10 200 $B --knob parallel_encoders=0 > $O/pip_ser_$r.json 2>> $O/err.txt
  timeout -k 10 200 $B --knob parallel_encoders=0 --no-pipeline > $O/seq_ser_$r.json 2>> $O/err.txt
  GPU_MAX_HW_QUEUES=8 timeout -k 10 200 $B > $O/pip_q8_$r.json 2>> $O/err.txt
  GPU_MAX_HW_QUEUES=8 timeout -k 10 200 $B --no-pipeline > $O/seq_q8_$r.json 2>> $O/err.txt
done
