#!/bin/bash
# Build libsfx plus the gemm2 experiment (gemm2.hip + the planes LayerNorm of norm_planes.patch) into
# experiments/gemm2/libsfx_gemm2.so; use it with SFX_LIB=experiments/gemm2/libsfx_gemm2.so.
set -e
cd "$(dirname "$0")/../.."
python -m splatformer_amd.build_lib > /dev/null
B=build/exp_gemm2
mkdir -p $B
cp splatformer_amd/csrc/norm.hip $B/norm.hip
(cd $B && patch -s -p3 < ../../experiments/gemm2/norm_planes.patch)
F="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=fast-honor-pragmas -munsafe-fp-atomics -Wno-unused-result -Isplatformer_amd/csrc -Iinclude"
/opt/rocm/bin/hipcc $F -c experiments/gemm2/gemm2.hip -o $B/gemm2.o
/opt/rocm/bin/hipcc $F -c $B/norm.hip -o $B/norm.o
objs=$(for f in splatformer_amd/csrc/*.hip; do b=$(basename $f .hip); [ $b = norm ] || echo build/sfx/$b.o; done)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs $B/gemm2.o $B/norm.o -o experiments/gemm2/libsfx_gemm2.so
echo built experiments/gemm2/libsfx_gemm2.so
