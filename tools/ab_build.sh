#!/bin/bash
# Build libdmf_hip.so variants for an interleaved A/B on the GPU box:
#   bash tools/ab_build.sh NAME [REV]   -> ab/NAME.so from csrc at git REV (default: working tree)
# Run them with DMF_HIP_LIB=ab/NAME.so (dmf_native honours it).
set -e
NAME=${1:?name}; REV=${2:-}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$(ls -d "$ROOT"/deep-multimodal-*_amd)
SRC=/tmp/ab_src_$NAME; rm -rf $SRC; mkdir -p $SRC/pkg/csrc $SRC/include
if [ -n "$REV" ]; then
  (cd "$ROOT" && git archive "$REV" "$(basename "$PKG")/csrc" include) | tar -x -C $SRC
  mv $SRC/$(basename "$PKG")/csrc/* $SRC/pkg/csrc/
else
  cp "$PKG"/csrc/*.hip "$PKG"/csrc/*.h "$PKG"/csrc/Makefile $SRC/pkg/csrc/; cp "$ROOT"/include/*.h $SRC/include/
fi
mkdir -p "$ROOT/ab"
make -C $SRC/pkg/csrc -j8 OUT="$ROOT/ab/$NAME.so" BUILD=$SRC/build > /tmp/ab_build_$NAME.log 2>&1 || { tail -20 /tmp/ab_build_$NAME.log; exit 1; }
echo "built ab/$NAME.so"
