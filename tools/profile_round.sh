#!/bin/bash
# Round profiling recipe (run on the GPU box from the repo root):
#   tools/profile_round.sh [label ...]      (default: every bench workload)
# Labels: config3 (the default bench job: 64 GiB of 32 KiB text streams, 8 GiB
# launches), text32k (configs[1], 1 GiB), text64k, random, repeat, decode10g.
# For each label W, under gpurun_out/prof/W/:
#   bench.json    the bench.py line (CPU baselines on a bounded sample)
#   trace/        rocprofv3 --kernel-trace --stats of the same command
#   fetch/ write/ rocprofv3 --pmc FETCH_SIZE, WRITE_SIZE (separate passes, kernel trace only)
#   sq/ sq2/      rocprofv3 --pmc of 8 + 8 SQ counters (instruction mix, wave cycles,
#                 issue / wait / LDS cycles: the busy fractions of DESIGN.md 4.2-4.3)
# tools/pmc_summary.py then writes profiles/<round>_W_*.  Every GPU step has its
# own time limit; steps are chained with && so the first failure ends the run.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
WLS=${*:-"config3 text32k text64k random repeat decode10g"}
STEPS=${STEPS:-5}
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"
SQ2="SQ_WAVES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD"
run() {  # workload
    # --no-sub: the profiled process runs this workload only (the default line also runs the
    # other configs, whose launches of the same kernels would be averaged into W's counters)
    local w=$1 d=gpurun_out/prof/$1 sel
    case $w in
        config3) sel="--workload text32k" ;;
        text32k) sel="--workload text32k --bytes-per-gpu 1073741824" ;;
        *) sel="--workload $w" ;;
    esac
    local q="$sel --no-cpu-baseline --no-host-e2e --no-sub"
    mkdir -p $d &&
    echo "[$(date +%T)] $w: bench" &&
    timeout -k 10 400 python3 bench.py $sel --steps $STEPS --warmup 2 --cpu-sample-bytes 268435456 --no-sub \
        > $d/bench.json 2> $d/bench.err &&
    echo "[$(date +%T)] $w: kernel trace" &&
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $d/trace -o run --output-format csv -- \
        python3 bench.py $q --steps $STEPS --warmup 2 > $d/trace.log 2>&1 &&
    echo "[$(date +%T)] $w: FETCH_SIZE" &&
    timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $d/fetch -o run --output-format csv -- \
        python3 bench.py $q --steps 2 --warmup 1 > $d/fetch.log 2>&1 &&
    echo "[$(date +%T)] $w: WRITE_SIZE" &&
    timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $d/write -o run --output-format csv -- \
        python3 bench.py $q --steps 2 --warmup 1 > $d/write.log 2>&1 &&
    echo "[$(date +%T)] $w: SQ counters" &&
    timeout -k 10 400 rocprofv3 --pmc $SQ --kernel-trace -d $d/sq -o run --output-format csv -- \
        python3 bench.py $q --steps 2 --warmup 1 > $d/sq.log 2>&1 &&
    echo "[$(date +%T)] $w: SQ counters, pass 2" &&
    timeout -k 10 400 rocprofv3 --pmc $SQ2 --kernel-trace -d $d/sq2 -o run --output-format csv -- \
        python3 bench.py $q --steps 2 --warmup 1 > $d/sq2.log 2>&1
}
for w in $WLS; do
    run $w || exit 1
done
echo "[$(date +%T)] done"
