#!/bin/bash
# Build an experiment variant of libtrajmpc.so under _variants/<name>/ with extra
# compiler flags (e.g. -DTGMPC_DPP_BC=1); tools/r04_iter.sh VARIANTS="<name> ..." benches it beside the in-tree
# library (TRAJMPC_LIB).  Usage: tools/build_variant.sh <name> <flags...>
set -e
cd "$(dirname "$0")/.."
name=$1; shift
make -s -j8 -C trajectory_generation_amd/csrc OUT=../../_variants/$name/libtrajmpc.so OBJDIR=../../_variants/$name/obj EXTRA="$*"
