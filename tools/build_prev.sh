#!/bin/bash
# Build the kernels of a git revision (default HEAD) into
# lightweight-snappy_amd/variants/libsnappy_amd_<name>.so (default name: prev)
# for A/B against the working tree with tools/variant_bench.py.  Same
# compile flags as the Makefile (compress kernels with the compress
# scheduler, decode kernels with max-ilp); host code from the working tree.
#   tools/build_prev.sh [REV] [NAME] [extra -D flags...]
set -e
cd "$(dirname "$0")/.."
REV=${1:-HEAD}
NAME=${2:-prev}
shift 2 2>/dev/null || shift $#
P=lightweight-snappy_amd
mkdir -p $P/variants $P/build
SRC=$P/csrc/.${NAME}_kernels.hip
if [ "$REV" = "WORK" ]; then cp $P/csrc/snappy_kernels.hip $SRC; else git show $REV:$P/csrc/snappy_kernels.hip > $SRC; fi
trap 'rm -f $SRC' EXIT
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -mcode-object-version=5 -Iinclude -I$P/csrc $*"
SC="-mllvm -amdgpu-sched-strategy=max-memory-clause -mllvm -amdgpu-use-amdgpu-trackers"
SD="-mllvm -amdgpu-sched-strategy=max-ilp"
hipcc $FLAGS $SC -DSNAPPY_TU=1 -x hip -c $SRC -o $P/build/kc_$NAME.o
hipcc $FLAGS $SD -DSNAPPY_TU=2 -x hip -c $SRC -o $P/build/kd_$NAME.o
hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -mcode-object-version=5 -Iinclude -I$P/csrc -c $P/csrc/snappy_device.hip -o $P/build/dev_var.o
gcc -O2 -fPIC -std=gnu11 -Iinclude -c $P/csrc/snappy_host.c -o $P/build/host_var.o
hipcc --offload-arch=gfx950 -shared -fPIC -o $P/variants/libsnappy_amd_$NAME.so $P/build/kc_$NAME.o $P/build/kd_$NAME.o \
    $P/build/dev_var.o $P/build/host_var.o
echo "built $NAME ($REV $*)"
