#!/bin/bash
# Round profiling recipe (run on the GPU box from the repo root):
#   1. bench.py default line                    -> gpurun_out/bench.json
#   2. rocprofv3 --kernel-trace --stats, same command  -> gpurun_out/prof_trace/
#   3. rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE (separate passes, kernel trace only)
# Each GPU step has its own time limit; steps are chained with &&.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-5}
timeout -k 10 400 python bench.py --steps $STEPS --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace -o run --output-format csv -- \
    python3 bench.py --steps $STEPS --warmup 2 --no-cpu-baseline --no-host-e2e > gpurun_out/prof_trace.log 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/prof_fetch -o run --output-format csv -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-e2e > gpurun_out/prof_fetch.log 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/prof_write -o run --output-format csv -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-e2e > gpurun_out/prof_write.log 2>&1
