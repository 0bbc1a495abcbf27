#!/bin/bash
# diagnostic builds of libamh.so with the d = 64 step kernel's variant switches
# (lib/var_<name>/libamh.so); select one at run time with AMH_LIB_PATH
set -e
cd "$(dirname "$0")/../adaptive-mcmc_amd/csrc"
OUT=../lib
FLAGS="--offload-arch=gfx950 -O3 -std=c++20 -fPIC -ffp-contract=off -fno-fast-math -fno-slp-vectorize -munsafe-fp-atomics -mllvm -amdgpu-atomic-optimizer-strategy=None"
for v in "$@"; do
  name=${v%%:*}; defs=${v#*:}
  mkdir -p $OUT/var_$name
  /opt/rocm/bin/hipcc $FLAGS $defs -c amh_kernels.hip -o $OUT/var_$name/k.o
  objs=$(ls $OUT/*.o | grep -v amh_kernels.o)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/var_$name/libamh.so $OUT/var_$name/k.o $objs
  echo built $name
done
