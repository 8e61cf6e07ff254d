#!/bin/bash
# Round 6: nontemporal output stores of the persistent 1x1 form (>= 100 MiB outputs), A/B on mode B,
# config 5 and config 2.
set -e
O=gpurun_out/r06p; mkdir -p $O
B="python bench.py --steps 20 --warmup 3 --no-extras --no-roofline --no-cpu-baseline"
for r in 1 2; do
  for t in 0 100; do
    timeout -k 10 200 $B --mode B --knob conv_nt_store_mb=$t > $O/b_nt${t}_$r.json 2>> $O/err.txt
    timeout -k 10 200 $B --config 5 --knob conv_nt_store_mb=$t > $O/c5_nt${t}_$r.json 2>> $O/err.txt
    timeout -k 10 200 $B --config 2 --knob conv_nt_store_mb=$t > $O/c2_nt${t}_$r.json 2>> $O/err.txt
  done
done
