#!/bin/bash
# Variant library for same-box A/B: csrc/var_NAME/libimls_gpu.so = project.hip built with extra
# flags (or from another source file, SRC=...) linked with the product's other objects.
# usage: tools/build_variant.sh NAME [-DFLAG=VALUE ...]
set -eu
C=planetary-lidar-odometry_amd/csrc
name=$1; shift
d=$C/var_$name
mkdir -p $d
src=${SRC:-$C/project.hip}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize -Wall \
    -Wno-unused-result -Wno-unused-value -I$C "$@" -c $src -o $d/project.o
objs=""
for o in index tv solve ransac normals scanreg front sample api; do objs="$objs $C/$o.o"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $d/libimls_gpu.so $d/project.o $objs
echo "built $d/libimls_gpu.so"
