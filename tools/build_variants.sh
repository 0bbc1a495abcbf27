#!/bin/bash
# diagnostic builds of libamh.so with compile-time switches of one source
# file: tools/build_variants.sh SRC "name:-DFLAG ..." ... -> lib/var_<name>/libamh.so
# (select one at run time with AMH_LIB_PATH)
set -e
cd "$(dirname "$0")/../adaptive-mcmc_amd/csrc"
SRC=$1; shift
OUT=../lib
FLAGS="--offload-arch=gfx950 -O3 -std=c++20 -fPIC -ffp-contract=off -fno-fast-math -fno-slp-vectorize -munsafe-fp-atomics -mllvm -amdgpu-atomic-optimizer-strategy=None"
base=$(basename $SRC .hip)
for v in "$@"; do
  name=${v%%:*}; defs=${v#*:}
  mkdir -p $OUT/var_$name
  /opt/rocm/bin/hipcc $FLAGS $defs -c $SRC -o $OUT/var_$name/v.o
  objs=$(ls $OUT/*.o | grep -v "/$base.o")
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/var_$name/libamh.so $OUT/var_$name/v.o $objs
  echo built $name
done
