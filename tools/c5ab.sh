#!/bin/bash
# Config 5 (S=384) conv-tile A/B: dump the step's conv shapes, time them per variant, then A/B whole steps.
#   bash tools/c5ab.sh   (on the GPU box; writes gpurun_out/c5/)
set -o pipefail
mkdir -p gpurun_out/c5
DMF_CONV_DUMP=gpurun_out/c5/conv.jsonl timeout -k 10 400 python bench.py --config 5 --no-cpu-baseline --no-extras --steps 10 --warmup 3 > gpurun_out/c5/bench.json 2> gpurun_out/c5/bench.err || { echo "bench failed"; tail -20 gpurun_out/c5/bench.err; exit 1; }
tail -c 400 gpurun_out/c5/bench.json
timeout -k 10 400 python tools/conv_bench.py --from gpurun_out/c5/conv.jsonl --tunes "15:256;15:289,14:256;7:0" --rounds 3 > gpurun_out/c5/ab.txt 2>&1 || { echo "conv ab failed"; tail -20 gpurun_out/c5/ab.txt; exit 1; }
cat gpurun_out/c5/ab.txt
AB_ARGS="--config 5 --no-roofline" timeout -k 10 900 bash tools/ab_env.sh 2 "-" "conv_sq_min_tiles=289" "conv_pp_mode=0"
