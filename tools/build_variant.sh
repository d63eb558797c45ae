#!/bin/sh
# build_variant.sh NAME "-DFOO=1 ..." [SRC [REPLACES]] — libppo with csrc/SRC.hip (default gemm) compiled
# under extra defines in place of csrc/REPLACES.hip (default SRC), for A/B sweeps and diagnostics on the GPU box (tools/*.py --lib
# ppo.c_amd/lib/variants/libppo_NAME.so); e.g. `build_variant.sh diag -DPPO_X3_DIAG gemm_x3`
set -e
cd "$(dirname "$0")/../ppo.c_amd"
SRC=${3:-gemm}
REP=${4:-$SRC}
mkdir -p build/variants lib/variants
HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function"
[ "$REP" = gemm_x3 ] && HIPFLAGS="$HIPFLAGS -fno-slp-vectorize"
/opt/rocm/bin/hipcc $HIPFLAGS $2 -c csrc/$SRC.hip -o build/variants/${SRC}_$1.o
OBJS=$(ls build/*.o | grep -v "build/$REP.hip.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -o lib/variants/libppo_$1.so $OBJS build/variants/${SRC}_$1.o -shared \
    -L/opt/rocm/lib -Wl,-rpath,/opt/rocm/lib -lrccl -Wl,--version-script=build/exports.map
