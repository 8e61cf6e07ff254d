#!/bin/bash
# Interleaved A/B of library builds (one process per run; rounds outer, builds inner): conv_bench on the
# hot pp shapes under each libdmf_pp_<tag>.so next to the product library.
# usage: LIBS="v01 v11" ROUNDS=3 bash tools/lib_ab.sh
set -o pipefail
PKG=deep-multimodal-fusion-of-dce-mri-and-dwi-for-automated-breast-tumor-classification-w.-foundation_amd
S=${S:-"32,32,32,512,512,3,1,4;128,32,32,2048,2048,1,1,1;32,32,32,3072,256,3,1,1;32,32,32,256,256,3,1,2;32,32,32,256,256,3,1,1"}
TUNES=${TUNES:-"7:2,15:128"}
for r in $(seq ${ROUNDS:-3}); do
  for v in $LIBS; do
    DMF_HIP_LIB=$(pwd)/$PKG/libdmf_pp_$v.so timeout -k 10 200 python3 tools/conv_bench.py --acc --shapes "$S" \
      --rounds 1 --reps 10 --tunes "$TUNES" | grep -v variants | sed "s/^/$v r$r /" || exit 1
  done
done
