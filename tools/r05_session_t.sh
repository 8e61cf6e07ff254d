#!/bin/bash
# r05t: the tile threshold inside the two-encoder fork (knob conc_min_tiles), persistent cap off.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/enc_fwd_ab.py --tunes "conc_min_tiles=128,conc_persist=0;conc_min_tiles=96,conc_persist=0;conc_min_tiles=64,conc_persist=0;conc_min_tiles=32,conc_persist=0;conc_min_tiles=64,conc_persist=192" --rounds 5 > gpurun_out/r05t_enc_ab2.txt 2>&1 || exit 1
grep variant gpurun_out/r05t_enc_ab2.txt
