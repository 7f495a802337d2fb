#!/bin/bash
# Build timing-comparison libraries in-tree (they travel to the GPU box with the snapshot):
#   tools/build_variant.sh base [REV]        -> shs_gpu/libshs_base.so from git revision REV (default HEAD~1)
#   tools/build_variant.sh NAME "-DFLAG ..."  -> shs_gpu/libshs_NAME.so from the working tree with extra flags
# Load one with SHS_GPU_LIB (tools/exp_variants.sh, tools/gpu_ab.sh).
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/leisure-software-renderer_amd
name=$1
if [ "$name" = base ]; then
  rev=${2:-HEAD~1}
  d=$(mktemp -d /tmp/shs_base_XXXX)
  git -C "$ROOT" archive "$rev" leisure-software-renderer_amd include | tar -x -C "$d"
  make -s -j8 -C "$d/leisure-software-renderer_amd" OUT="$PKG/shs_gpu/libshs_base.so" OBJDIR="$d/obj"
  rm -rf "$d"
else
  make -s -j8 -C "$PKG" OUT="shs_gpu/libshs_$name.so" OBJDIR="build/obj_$name" EXTRA="$2"
fi
