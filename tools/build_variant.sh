#!/bin/bash
# Builds a library variant for A/B timing (tools/ab_gn.sh): variants/libpba_<name>.so from the same sources with extra
# compile definitions, in an object directory of its own.  Usage: tools/build_variant.sh <name> [-DFOO ...]
set -eu
cd "$(dirname "$0")/../photometric-bundle-adjustment_amd/csrc"
name=$1; shift
FL="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-result $*"
mkdir -p ../../variants
objs=$(make -s -j8 OBJDIR=obj_$name FLAGS="$FL" -pn 2>/dev/null | sed -n 's/^OBJS := //p' | head -1)
make -s -j8 OBJDIR=obj_$name FLAGS="$FL" $objs
/opt/rocm/bin/hipcc $FL -shared -o ../../variants/libpba_$name.so $objs -ldl
