#!/bin/bash
# Debug / experiment variant of the library: tools/build_variant.sh NAME "-DFLAG ..." builds every
# kernel with the extra flags into tools/bin/v/NAME/ and links tools/bin/v/libNAME.so (select it with
# PLAINCV_HIP_LIB=...; tools/bin/ is git-ignored but travels to the GPU box; the objects do not).
set -e
NAME=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
make -C $R/plaincv_amd/csrc -j${MAKE_JOBS:-8} OBJDIR=$R/tools/bin/v/$NAME LIB=$R/tools/bin/v/lib$NAME.so EXTRA="$*" >/dev/null
echo $R/tools/bin/v/lib$NAME.so
