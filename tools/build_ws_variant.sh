#!/bin/bash
# Experimental libsfx variant with extra flags for gemm_ws.hip only:
#   tools/build_ws_variant.sh <name> <extra hipcc flags...>   -> splatformer_amd/exp_<name>.so (SFX_LIB=...)
set -e
cd "$(dirname "$0")/.."
name=$1; shift
mkdir -p build/exp_$name
for f in splatformer_amd/csrc/*.hip; do
  b=$(basename $f .hip)
  if [ $b = gemm_ws ]; then
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=fast-honor-pragmas -munsafe-fp-atomics \
      -Wno-unused-result -Isplatformer_amd/csrc -Iinclude "$@" -c $f -o build/exp_$name/gemm_ws.o
  else
    cp build/sfx/$b.o build/exp_$name/
  fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC build/exp_$name/*.o -o splatformer_amd/exp_$name.so
echo built splatformer_amd/exp_$name.so
