#!/bin/bash
# VGPR / SGPR / spill counts of the K1r kernels in a build object (default the
# in-tree compress object; e.g. lightweight-snappy_amd/build/kc_<variant>.o)
set -e
obj=${1:-lightweight-snappy_amd/build/snappy_kernels_c.o}
t=$(mktemp -d)
objcopy --dump-section=.hip_fatbin=$t/fat.bin "$obj" $t/copy.o
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=$t/fat.bin \
    --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$t/k.co
/opt/rocm/lib/llvm/bin/llvm-readobj --notes $t/k.co | python3 "$(dirname "$0")/kres.py"
rm -rf $t
