#!/bin/bash
# Variant library for same-box A/B built from EVERY source with extra flags (flags that change a
# layout shared between files, e.g. -DIMLS_FINISH_QUAD=0 and the pass-1 slab size, need this; a
# project.hip-only flag can use tools/build_variant.sh): csrc/var_NAME/libimls_gpu.so.
# usage: tools/build_full_variant.sh NAME [-DFLAG=VALUE ...]
set -eu
C=planetary-lidar-odometry_amd/csrc
name=$1; shift
make -s -C $C variant VARIANT_FLAGS="$*" -j8
rm -rf $C/var_$name
mv $C/variant $C/var_$name
echo "built $C/var_$name/libimls_gpu.so"
