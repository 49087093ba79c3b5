#!/bin/bash
# Build the kernels of a git revision (default HEAD) into
# lightweight-snappy_amd/variants/libsnappy_amd_prev.so for A/B against the
# working tree with tools/variant_bench.py (host code from the working tree).
set -e
cd "$(dirname "$0")/.."
REV=${1:-HEAD}
P=lightweight-snappy_amd
mkdir -p $P/variants $P/build
git show $REV:$P/csrc/snappy_kernels.hip > $P/csrc/.prev_kernels.hip
trap 'rm -f $P/csrc/.prev_kernels.hip' EXIT
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -mcode-object-version=5 -Iinclude -I$P/csrc -mllvm -amdgpu-sched-strategy=max-ilp"
hipcc $FLAGS -x hip -c $P/csrc/.prev_kernels.hip -o $P/build/k_prev.o
hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -mcode-object-version=5 -Iinclude -I$P/csrc -c $P/csrc/snappy_device.hip -o $P/build/dev_var.o
gcc -O2 -fPIC -std=gnu11 -Iinclude -c $P/csrc/snappy_host.c -o $P/build/host_var.o
hipcc --offload-arch=gfx950 -shared -fPIC -o $P/variants/libsnappy_amd_prev.so $P/build/k_prev.o $P/build/dev_var.o $P/build/host_var.o
echo "built prev ($REV)"
