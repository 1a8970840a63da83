#!/bin/bash
# Debug / experiment variant of the library: tools/build_variant.sh NAME "-DFLAG ..." builds every
# kernel with the extra flags into scratch/v/NAME/ and links scratch/v/libNAME.so (select it with
# PLAINCV_HIP_LIB=...; scratch/ is git-ignored but travels to the GPU box).
set -e
NAME=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
make -C $R/plaincv_amd/csrc -j${MAKE_JOBS:-8} OBJDIR=$R/scratch/v/$NAME LIB=$R/scratch/v/lib$NAME.so EXTRA="$*" >/dev/null
echo $R/scratch/v/lib$NAME.so
