#!/bin/bash
# Placement-sweep builds of the working tree: the decode TU and the host
# objects once, the compress TU once per variant (NAME:-D flags ...), into
# lightweight-snappy_amd/variants/libsnappy_amd_<NAME>.so for tools/variant_bench.py.
#   tools/build_pads.sh 'a2:-DSNAPPY_K1R_PAD32=2' 'e2:-DSNAPPY_K1R_WIN_ENT=0 -DSNAPPY_K1R_PAD32=2' ...
# (env BASE: -D flags every variant gets)
set -e
cd "$(dirname "$0")/.."
P=lightweight-snappy_amd; B=$P/build; mkdir -p $P/variants
make -s -C $P >/dev/null  # the host objects of the tree
FL="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -mcode-object-version=5 -Iinclude -I$P/csrc"
SC="-mllvm -amdgpu-sched-strategy=max-memory-clause -mllvm -amdgpu-use-amdgpu-trackers"
SD="-mllvm -amdgpu-sched-strategy=max-ilp -mllvm -amdgpu-use-amdgpu-trackers"
hipcc $FL $SD $BASE -DSNAPPY_TU=2 -c $P/csrc/snappy_kernels.hip -o $B/pad_kd.o
hipcc $FL $BASE -c $P/csrc/snappy_device.hip -o $B/pad_dev.o
build_one() {
    local name=${1%%:*} defs=${1#*:}
    hipcc $FL $SC $BASE $defs -DSNAPPY_TU=1 -c $P/csrc/snappy_kernels.hip -o $B/pad_kc_$name.o
    hipcc --offload-arch=gfx950 -shared -fPIC -o $P/variants/libsnappy_amd_$name.so $B/pad_kc_$name.o $B/pad_kd.o \
        $B/pad_dev.o $B/snappy_pipeline.o $B/snappy_host.o $B/bst_host.o
    echo "built $name ($defs)"
}
# four compiles at a time
n=0
for spec in "$@"; do
    build_one "$spec" &
    n=$((n + 1))
    if [ $((n % 4)) -eq 0 ]; then wait; fi
done
wait
