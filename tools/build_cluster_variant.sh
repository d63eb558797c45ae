#!/bin/sh
# build_cluster_variant.sh NAME "DEFINES" [GIT-REV] — libppo with csrc/cluster.hip and csrc/cluster_deep.hip
# (from the working tree, or as of GIT-REV) compiled under extra defines, for same-box A/Bs of the
# B = 64 phases: ppo.c_amd/lib/variants/libppo_NAME.so
set -e
cd "$(dirname "$0")/../ppo.c_amd"
mkdir -p build/variants/src_$1 lib/variants
for f in cluster.hip cluster_deep.hip cluster_common.h; do
  if [ -n "$3" ]; then git show "$3:ppo.c_amd/csrc/$f" > build/variants/src_$1/$f; else cp csrc/$f build/variants/src_$1/$f; fi
done
HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function -Icsrc"
for f in cluster cluster_deep; do
  /opt/rocm/bin/hipcc $HIPFLAGS $2 -c build/variants/src_$1/$f.hip -o build/variants/${f}_$1.o
done
OBJS=$(ls build/*.o | grep -v "build/cluster.hip.o" | grep -v "build/cluster_deep.hip.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -o lib/variants/libppo_$1.so $OBJS build/variants/cluster_$1.o \
    build/variants/cluster_deep_$1.o -shared -L/opt/rocm/lib -Wl,-rpath,/opt/rocm/lib -lrccl -Wl,--version-script=build/exports.map
