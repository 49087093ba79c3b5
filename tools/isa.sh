#!/bin/bash
# Device ISA and per-kernel resources of snappy_kernels.hip (build container):
#   tools/isa.sh [extra hipcc flags]  -> /tmp/isa/k.s, resource table on stdout
set -e
cd "$(dirname "$0")/.."
mkdir -p /tmp/isa
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -mcode-object-version=5 --offload-device-only \
    -mllvm -amdgpu-sched-strategy=max-ilp -Iinclude -Ilightweight-snappy_amd/csrc "$@" \
    -c lightweight-snappy_amd/csrc/snappy_kernels.hip -o /tmp/isa/k.bundle
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=/tmp/isa/k.bundle \
    --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=/tmp/isa/k.co
/opt/rocm/lib/llvm/bin/llvm-objdump -d /tmp/isa/k.co > /tmp/isa/k.s
/opt/rocm/lib/llvm/bin/llvm-readobj --notes /tmp/isa/k.co | python3 tools/kres.py
