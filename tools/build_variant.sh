#!/bin/bash
# Build an experimental libsfx variant with extra hipcc flags for one source (default gemm.hip):
#   [SRC=gemm2] tools/build_variant.sh <name> <extra hipcc flags...>   -> splatformer_amd/exp_<name>.so (SFX_LIB=...)
set -e
cd "$(dirname "$0")/.."
python -m splatformer_amd.build_lib > /dev/null
SRC=${SRC:-gemm}
name=$1; shift
mkdir -p build/exp_$name
for f in splatformer_amd/csrc/*.hip; do
  b=$(basename $f .hip)
  if [ $b = $SRC ]; then
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=fast-honor-pragmas -munsafe-fp-atomics \
      -Wno-unused-result -Isplatformer_amd/csrc -Iinclude "$@" -c $f -o build/exp_$name/$b.o
  else
    cp build/sfx/$b.o build/exp_$name/
  fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC build/exp_$name/*.o -o splatformer_amd/exp_$name.so
echo built splatformer_amd/exp_$name.so
