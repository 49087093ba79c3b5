#!/bin/bash
# Build experimental kernel variants (compile-time knobs) into
# lightweight-snappy_amd/variants/ for A/B timing with tools/variant_bench.py.
set -e
cd "$(dirname "$0")/.."
PKG=lightweight-snappy_amd
mkdir -p $PKG/variants $PKG/build
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -mcode-object-version=5 -Iinclude -I$PKG/csrc"
KFLAGS=${KFLAGS-"-mllvm -amdgpu-sched-strategy=max-ilp"}  # as the Makefile (override: KFLAGS=...)
gcc -O2 -fPIC -std=gnu11 -Iinclude -c $PKG/csrc/snappy_host.c -o $PKG/build/host_var.o
g++ -O2 -std=c++17 -fPIC -pthread -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude -I$PKG/csrc \
    -c $PKG/csrc/snappy_pipeline.cpp -o $PKG/build/pipe_var.o
for spec in "$@"; do
  name=${spec%%:*}; defs=${spec#*:}
  # the device shim too: launch geometry knobs (SNAPPY_K2_SEG, ...) are shared with it
  hipcc $FLAGS $defs -c $PKG/csrc/snappy_device.hip -o $PKG/build/dev_$name.o
  hipcc $FLAGS $KFLAGS $defs -c $PKG/csrc/snappy_kernels.hip -o $PKG/build/k_$name.o
  hipcc --offload-arch=gfx950 -shared -fPIC -o $PKG/variants/libsnappy_amd_$name.so $PKG/build/k_$name.o $PKG/build/dev_$name.o $PKG/build/pipe_var.o $PKG/build/host_var.o
  echo "built $name ($defs)"
done
