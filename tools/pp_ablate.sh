#!/bin/bash
# K-loop ablation of the ping-pong conv (k_conv_fwd_pp): libraries whose conv_pp.o was compiled with
# -DDMF_PP_ABLATE=<bits> (bit 1 skips the steady state's vmcnt waits, 2 its LDS-DMA issue, 4 its fragment
# reads, 8 its MFMAs; outputs are garbage under any bit), built next to the product library as
# libdmf_pp_abl<bits>.so. Timing only, one process per library (pp forced, 128-tile launches allowed).
set -o pipefail
PKG=deep-multimodal-fusion-of-dce-mri-and-dwi-for-automated-breast-tumor-classification-w.-foundation_amd
S=${S:-"32,32,32,512,512,3,1,4;128,32,32,2048,2048,1,1,1;32,32,32,3072,256,3,1,1;32,32,32,256,256,3,1,2"}
for v in ${VARIANTS:-0 3 7 15}; do
  echo "== DMF_PP_ABLATE=$v"
  DMF_HIP_LIB=$(pwd)/$PKG/libdmf_pp_abl$v.so timeout -k 10 200 python3 tools/conv_bench.py --acc --shapes "$S" \
    --rounds 3 --reps 10 --tunes "7:2,15:128" | grep -v variants || exit 1
done
