#!/bin/sh
# build_variant.sh NAME "-DFOO=1 ..." — libppo with gemm.hip compiled under extra defines, for A/B
# sweeps on the GPU box (tools/gemm_sweep.py --lib ppo.c_amd/lib/variants/libppo_NAME.so)
set -e
cd "$(dirname "$0")/.."
mkdir -p build/variants lib/variants
HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function"
/opt/rocm/bin/hipcc $HIPFLAGS $2 -c csrc/gemm.hip -o build/variants/gemm_$1.o
OBJS=$(ls build/*.o | grep -v "build/gemm.hip.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -o lib/variants/libppo_$1.so $OBJS build/variants/gemm_$1.o -shared \
    -L/opt/rocm/lib -Wl,-rpath,/opt/rocm/lib -lrccl -Wl,--version-script=build/exports.map
