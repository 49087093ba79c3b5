#!/bin/bash
# Build the kernels of a git revision (default HEAD) into
# lightweight-snappy_amd/variants/libsnappy_amd_<name>.so (default name: prev)
# for A/B against the working tree with tools/variant_bench.py.  Same
# compile flags as the Makefile (compress kernels with the compress
# scheduler, decode kernels with max-ilp); kernels + device shim from REV,
# the C host code from the working tree.
#   tools/build_prev.sh [REV|WORK|DIR:path] [NAME] [extra -D flags...]
set -e
cd "$(dirname "$0")/.."
REV=${1:-HEAD}
NAME=${2:-prev}
shift 2 2>/dev/null || shift $#
P=lightweight-snappy_amd
mkdir -p $P/variants $P/build
# the kernels, their private header and the device shim from REV (the
# shim launches the kernels with REV's signatures); the C host from the tree
D=$P/build/src_$NAME
rm -rf $D && mkdir -p $D
# (from round 5 the shim's host pipelines are snappy_pipeline.cpp + snappy_ctx.h;
# older revisions hold them in snappy_device.hip, so those two may be absent)
for f in snappy_kernels.hip snappy_kernels.h snappy_device.hip snappy_ctx.h snappy_pipeline.cpp; do
    case $REV in
    WORK) [ -f $P/csrc/$f ] && cp $P/csrc/$f $D/$f ;;
    DIR:*) [ -f ${REV#DIR:}/$f ] && cp ${REV#DIR:}/$f $D/$f ;;  # a directory holding the files
    *) git show $REV:$P/csrc/$f > $D/$f 2>/dev/null || rm -f $D/$f ;;
    esac
done
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=${VARCH:-gfx950} -mcode-object-version=5 -Iinclude -I$D $*"
SC=${SCHED_C-"-mllvm -amdgpu-sched-strategy=max-memory-clause -mllvm -amdgpu-use-amdgpu-trackers"}  # env SCHED_C overrides (A/B)
SD=${SCHED_D-"-mllvm -amdgpu-sched-strategy=max-ilp -mllvm -amdgpu-use-amdgpu-trackers"}
hipcc $FLAGS $SC -DSNAPPY_TU=1 -x hip -c $D/snappy_kernels.hip -o $P/build/kc_$NAME.o
hipcc $FLAGS $SD -DSNAPPY_TU=2 -x hip -c $D/snappy_kernels.hip -o $P/build/kd_$NAME.o
hipcc -O3 -std=c++17 -fPIC --offload-arch=${VARCH:-gfx950} -mcode-object-version=5 -Iinclude -I$D -c $D/snappy_device.hip -o $P/build/dev_$NAME.o
gcc -O2 -fPIC -std=gnu11 -Iinclude -c $P/csrc/snappy_host.c -o $P/build/host_var.o
PIPE=""
if [ -f $D/snappy_pipeline.cpp ]; then
    g++ -O2 -std=c++17 -fPIC -pthread -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude -I$D \
        -c $D/snappy_pipeline.cpp -o $P/build/pipe_$NAME.o
    PIPE=$P/build/pipe_$NAME.o
fi
# the working tree's -b compressor and weak stubs of newer entry points (tools/variant_stub.c)
gcc -O2 -fPIC -std=gnu11 -pthread -Iinclude -c $P/csrc/bst_host.c -o $P/build/bst_var.o
gcc -O2 -fPIC -std=gnu11 -Iinclude -c tools/variant_stub.c -o $P/build/stub_var.o
hipcc --offload-arch=${VARCH:-gfx950} -shared -fPIC -o $P/variants/libsnappy_amd_$NAME.so $P/build/kc_$NAME.o $P/build/kd_$NAME.o \
    $P/build/dev_$NAME.o $PIPE $P/build/host_var.o $P/build/bst_var.o $P/build/stub_var.o
rm -rf $D
echo "built $NAME ($REV $*)"
