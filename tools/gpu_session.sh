#!/bin/bash
# One GPU-box session of checks (run from the repo root on the box):
#   tools/gpu_session.sh <outdir> [tests] [bench] [n1_64g] [prof64g] [profile <workloads...>]
# Every GPU step has its own time limit; a step that times out, aborts or
# faults ends the session (exit codes 124/134/137/139 and signals), and a
# failing pytest run (rc 1) is recorded but does not stop the benches.
set -o pipefail
export TMPDIR=/tmp
out=${1:?outdir}; shift
mkdir -p "$out"
export SNAPPY_TEST_PROGRESS=$(cd "$out" && pwd)/test_progress.log
fatal() { case $1 in 0|1) return 1;; *) return 0;; esac; }
for step in "$@"; do
    echo "[$(date +%T)] $step"
    case $step in
    tests)
        timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
            > "$out/gpu_tests.log" 2>&1
        rc=$?; echo "tests rc=$rc"; tail -3 "$out/gpu_tests.log"
        fatal $rc && exit $rc ;;
    bench)
        timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > "$out/bench.json" 2> "$out/bench.err"
        rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && exit $rc ;;
    n1_64g)  # the N = 1 point of configs[3]: 64 GiB of 32 KiB text streams on one GPU
        timeout -k 10 600 python -u bench.py --total-bytes 68719476736 --steps 5 --warmup 1 \
            --cpu-sample-bytes 268435456 > "$out/n1_64g.json" 2> "$out/n1_64g.err"
        rc=$?; echo "n1_64g rc=$rc"; [ $rc -ne 0 ] && exit $rc ;;
    prof64g)
        timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$out/n1_64g_trace" -o run --output-format csv -- \
            python3 bench.py --total-bytes 68719476736 --steps 2 --warmup 1 --no-cpu-baseline --no-host-e2e \
            > "$out/n1_64g_trace.log" 2>&1
        rc=$?; echo "prof64g rc=$rc"; [ $rc -ne 0 ] && exit $rc ;;
    ovl)  # the default job with and without --overlap (decode of piece k during the compress of k + 1)
        for o in "" "--overlap" "" "--overlap"; do
            timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --no-sub --no-cpu-baseline --no-host-e2e $o \
                >> "$out/ovl.json" 2>> "$out/ovl.err"
            rc=$?; echo "ovl '$o' rc=$rc"; [ $rc -ne 0 ] && exit $rc
        done
        python3 -c "import json,sys; [print(d['config']['overlap'], d['ms_per_step'], d['value'], d['kernel_ms'], d['round_trip_ok']) for d in map(json.loads, [l for l in open(sys.argv[1]) if l.startswith('{')])]" "$out/ovl.json" ;;
    ab:*)  # ab:<variant,variant,...>:<kind>:<chunk>:<layout> -> tools/variant_bench.py, 1 GiB
        IFS=: read -r _ vs kind chunk layout <<< "$step"
        timeout -k 10 400 python -u tools/variant_bench.py ${vs//,/ } --kind $kind --n 1073741824 --chunk $chunk \
            --layout $layout --reps 3 --rounds 2 > "$out/ab_${vs//,/-}_${kind}_${chunk}.log" 2>&1
        rc=$?; echo "ab rc=$rc"; tail -6 "$out/ab_${vs//,/-}_${kind}_${chunk}.log"; [ $rc -ne 0 ] && exit $rc ;;
    pmc:*)  # pmc:<tag>:<workload>:<COUNTER,COUNTER,...> -> one rocprofv3 counter pass over a 1-step bench
        IFS=: read -r _ tag wl ctrs <<< "$step"
        timeout -s KILL 240 rocprofv3 --pmc ${ctrs//,/ } --kernel-trace -d "$out/pmc_$tag" -o run \
            --output-format csv -- python3 bench.py --workload $wl --steps 1 --warmup 1 --no-cpu-baseline \
            --no-host-e2e --no-sub > "$out/pmc_$tag.log" 2>&1
        rc=$?; echo "pmc $tag rc=$rc"; [ $rc -ne 0 ] && exit $rc ;;
    pmcv:*)  # pmcv:<variant>:<tag>:<workload>:<COUNTERS> -> the same pass over variants/libsnappy_amd_<variant>.so
        IFS=: read -r _ var tag wl ctrs <<< "$step"
        SNAPPY_AMD_LIB=$PWD/lightweight-snappy_amd/variants/libsnappy_amd_$var.so \
            timeout -s KILL 240 rocprofv3 --pmc ${ctrs//,/ } --kernel-trace -d "$out/pmc_$tag" -o run \
            --output-format csv -- python3 bench.py --workload $wl --steps 1 --warmup 1 --no-cpu-baseline \
            --no-host-e2e --no-sub > "$out/pmc_$tag.log" 2>&1
        rc=$?; echo "pmcv $tag rc=$rc"; [ $rc -ne 0 ] && exit $rc ;;
    counters)
        timeout -k 10 120 rocprofv3 --list-avail > "$out/counters.txt" 2>&1
        rc=$?; echo "counters rc=$rc"; [ $rc -ne 0 ] && exit $rc ;;
    occ:*)  # occ:<kind>:<chunk>:<dynlds,...> -> K1r statistics build at reduced occupancy
        IFS=: read -r _ kind chunk dyns <<< "$step"
        for d in ${dyns//,/ }; do
            SNAPPY_K1R_DYNLDS=$d timeout -k 10 200 python -u tools/k1r_stats.py $kind 268435456 $chunk \
                > "$out/occ_${kind}_${chunk}_$d.log" 2>&1
            rc=$?; echo "occ $d rc=$rc"; cat "$out/occ_${kind}_${chunk}_$d.log"; [ $rc -ne 0 ] && exit $rc
        done ;;
    k4s:*)  # k4s:<variant,...>:<kind> -> K4 statistics builds (SNAPPY_K4_STATS), 256 MiB of 32 KiB streams
        IFS=: read -r _ vs kind <<< "$step"
        for v in ${vs//,/ }; do
            timeout -k 10 200 python -u tools/k4_stats.py $kind 268435456 $v > "$out/k4s_${v}_$kind.log" 2>&1
            rc=$?; echo "k4s $v rc=$rc"; cat "$out/k4s_${v}_$kind.log"; [ $rc -ne 0 ] && exit $rc
        done ;;
    k1s:*)  # k1s:<variant>:<chunk>:<rounds per unit> -> K1r round segments (SNAPPY_K1R_STATS + LSTAMPS build), 256 MiB
        IFS=: read -r _ v chunk rnds <<< "$step"
        K1R_CHUNK=$chunk K1R_ROUNDS=$rnds timeout -k 10 200 python -u tools/k1r_stamps.py 268435456 "" $v \
            > "$out/k1s_${v}_$chunk.log" 2>&1
        rc=$?; echo "k1s $v rc=$rc"; cat "$out/k1s_${v}_$chunk.log"; [ $rc -ne 0 ] && exit $rc ;;
    pageable)  # host-buffer staging floor: runtime pageable copies vs threaded memcpy into pinned memory
        timeout -k 10 200 python -u tools/pageable_probe.py > "$out/pageable_probe.log" 2>&1
        rc=$?; echo "pageable rc=$rc"; cat "$out/pageable_probe.log"; [ $rc -ne 0 ] && exit $rc ;;
    ovl16)  # --overlap A/B at 16 GiB (two pieces)
        for o in "" "--overlap" "" "--overlap"; do
            timeout -k 10 300 python -u bench.py --total-bytes 17179869184 --steps 4 --warmup 1 --no-sub --no-cpu-baseline \
                --no-host-e2e $o >> "$out/ovl16.json" 2>> "$out/ovl16.err"
            rc=$?; echo "ovl16 '$o' rc=$rc"; [ $rc -ne 0 ] && exit $rc
        done
        python3 -c "import json,sys; [print(d['config']['overlap'], d['ms_per_step'], d['value'], d['kernel_ms'], d['round_trip_ok']) for d in map(json.loads, [l for l in open(sys.argv[1]) if l.startswith('{')])]" "$out/ovl16.json" ;;
    hostpipe)  # host-buffer compress pipeline: lanes x chunk MiB sweep (tools/host_e2e.py, text 256 MiB)
        for lc in 4:64 3:64 4:48 5:48 6:32 4:64; do
            SNAPPY_AMD_PIPE_LANES=${lc%%:*} SNAPPY_AMD_PIPE_CHUNK_MB=${lc##*:} timeout -k 10 120 \
                python -u tools/host_e2e.py 268435456 T > "$out/hostpipe_$lc.log" 2>&1
            rc=$?; echo "hostpipe $lc rc=$rc: $(grep -h '^T' "$out/hostpipe_$lc.log")"; [ $rc -ne 0 ] && exit $rc
        done ;;
    hostab:*)  # hostab:<variant,...> -> tools/host_e2e.py (text 256 MiB) per library variant, twice, interleaved
        vs=${step#hostab:}
        for r in 1 2; do for v in ${vs//,/ }; do
            lib=""; [ "$v" != default ] && lib=$PWD/lightweight-snappy_amd/variants/libsnappy_amd_$v.so
            SNAPPY_AMD_LIB=$lib timeout -k 10 120 python -u tools/host_e2e.py 268435456 T > "$out/hostab_${v}_$r.log" 2>&1
            rc=$?; echo "hostab $v rc=$rc: $(grep -h '^T' "$out/hostab_${v}_$r.log")"; [ $rc -ne 0 ] && exit $rc
        done; done ;;
    copypath)  # which copy path (DMA engines or blit kernels) pageable copies take per stream (tools/micro/copy_path.hip)
        timeout -k 10 120 tools/micro/copy_path > "$out/copy_path.log" 2>&1
        rc=$?; echo "copypath rc=$rc"; cat "$out/copy_path.log"; [ $rc -ne 0 ] && exit $rc ;;
    hostinbench)  # the bench line's host_end_to_end after a 1 GiB and after the 64 GiB job (no sub-results, no CPU baselines)
        for tb in 1073741824 68719476736; do
            timeout -k 10 400 python -u bench.py --total-bytes $tb --steps 2 --warmup 1 --no-sub --no-cpu-baseline \
                > "$out/hostinbench_$tb.json" 2> "$out/hostinbench_$tb.err"
            rc=$?; echo "hostinbench $tb rc=$rc: $(python3 -c "import json,sys; print(json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])['host_end_to_end'])" "$out/hostinbench_$tb.json")"
            [ $rc -ne 0 ] && exit $rc
        done
        timeout -k 10 500 rocprofv3 --kernel-trace --memory-copy-trace -d "$out/hostinbench_trace" -o run --output-format csv -- \
            python3 bench.py --steps 1 --warmup 1 --no-sub --no-cpu-baseline > "$out/hostinbench_trace.log" 2>&1
        rc=$?; echo "hostinbench trace rc=$rc"; [ $rc -ne 0 ] && exit $rc ;;
    hostenv)  # host_end_to_end inside a 1 GiB bench run: as is, with high-priority lane streams, with 8 hardware queues
        for e in ${HOSTENV_SET:-"X=1" "SNAPPY_AMD_PIPE_PRIO=1" "GPU_MAX_HW_QUEUES=8"}; do
            env $e timeout -k 10 300 python -u bench.py --total-bytes 1073741824 --steps 2 --warmup 1 --no-sub --no-cpu-baseline \
                > "$out/hostenv_$e.json" 2> "$out/hostenv_$e.err"
            rc=$?; echo "hostenv $e rc=$rc: $(python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(d['value'], d['host_end_to_end'])" "$out/hostenv_$e.json")"
            [ $rc -ne 0 ] && exit $rc
        done ;;
    hostenvab:*)  # hostenvab:<ENV=V+ENV=V,...> -> tools/host_e2e.py (text 256 MiB) per env set, twice, interleaved
        sets=${step#hostenvab:}
        for r in 1 2; do for e in ${sets//,/ }; do
            env ${e//+/ } timeout -k 10 120 python -u tools/host_e2e.py 268435456 T > "$out/hostenvab_${e}_$r.log" 2>&1
            rc=$?; echo "hostenvab $e rc=$rc: $(grep -h '^T' "$out/hostenvab_${e}_$r.log")"; [ $rc -ne 0 ] && exit $rc
        done; done ;;
    hosttraceenv:*)  # hosttraceenv:<ENV=V+...> -> kernel + memory-copy trace of tools/host_e2e.py under that env
        e=${step#hosttraceenv:}
        env ${e//+/ } timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d "$out/hosttraceenv" -o run \
            --output-format csv -- python3 tools/host_e2e.py 268435456 T > "$out/hosttraceenv.log" 2>&1
        rc=$?; echo "hosttraceenv rc=$rc"; [ $rc -ne 0 ] && exit $rc ;;
    fileab:*)  # fileab:<ENV=V+...,...> -> bench.host_file_api (4 GiB text in /dev/shm, IO trace) per env set, twice, interleaved
        sets=${step#fileab:}
        for r in 1 2; do for e in ${sets//,/ }; do
            env SNAPPY_AMD_IO_TRACE=1 ${e//+/ } timeout -k 10 200 python -u -c "import json, bench; print(json.dumps(bench.host_file_api(4 << 30)))" \
                > "$out/fileab_${e}_$r.log" 2>&1
            rc=$?; echo "fileab $e rc=$rc: $(grep -h 'compress_MBps' "$out/fileab_${e}_$r.log")"; [ $rc -ne 0 ] && exit $rc
        done; done ;;
    hostctxab)  # host context's own stream at default vs high priority: tools/host_e2e.py twice each, then a trace of the latter
        for r in 1 2; do for e in X=1 SNAPPY_AMD_HOSTCTX_PRIO=1; do
            env $e timeout -k 10 120 python -u tools/host_e2e.py 268435456 T > "$out/hostctxab_${e}_$r.log" 2>&1
            rc=$?; echo "hostctxab $e rc=$rc: $(grep -h '^T' "$out/hostctxab_${e}_$r.log")"; [ $rc -ne 0 ] && exit $rc
        done; done
        SNAPPY_AMD_HOSTCTX_PRIO=1 timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d "$out/hostctx_trace" -o run \
            --output-format csv -- python3 tools/host_e2e.py 268435456 T > "$out/hostctx_trace.log" 2>&1
        rc=$?; echo "hostctx trace rc=$rc"; [ $rc -ne 0 ] && exit $rc ;;
    benchv:*)  # benchv:<variant,...>:<workload> -> bench.py --workload W per library variant (no sub-results, CPU or host legs)
        IFS=: read -r _ vs wl <<< "$step"
        for v in ${vs//,/ }; do
            lib=""; [ "$v" != default ] && lib=$PWD/lightweight-snappy_amd/variants/libsnappy_amd_$v.so
            SNAPPY_AMD_LIB=$lib timeout -k 10 300 python -u bench.py --workload $wl --steps 5 --warmup 2 --no-sub \
                --no-cpu-baseline --no-host-e2e > "$out/benchv_${v}_$wl.json" 2> "$out/benchv_${v}_$wl.err"
            rc=$?; echo "benchv $v $wl rc=$rc: $(python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(d['value'], d['kernel_ms'])" "$out/benchv_${v}_$wl.json")"
            [ $rc -ne 0 ] && exit $rc
        done ;;
    hosttrace)  # kernel + memory-copy trace of the host-buffer API (timeline of the pipeline)
        timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$out/hosttrace" -o run \
            --output-format csv -- python3 tools/host_e2e.py 268435456 T > "$out/hosttrace.log" 2>&1
        rc=$?; echo "hosttrace rc=$rc"; [ $rc -ne 0 ] && exit $rc ;;
    io)  # host I/O floor (tools/io_probe.py, no GPU) and the FILE* API with SNAPPY_AMD_IO_TRACE phase times
        timeout -k 10 200 python -u tools/io_probe.py 4 > "$out/io_probe.log" 2>&1
        rc=$?; echo "io_probe rc=$rc"; cat "$out/io_probe.log"; [ $rc -ne 0 ] && exit $rc
        SNAPPY_AMD_IO_TRACE=1 timeout -k 10 300 python -u -c "import json, bench; print(json.dumps(bench.host_file_api(4 << 30)))" \
            > "$out/file_api.log" 2>&1
        rc=$?; echo "file_api rc=$rc"; tail -20 "$out/file_api.log"; [ $rc -ne 0 ] && exit $rc ;;
    pytest:*)  # pytest:<-k expression, "_or_" for " or "> -> the GPU tests it selects
        expr=${step#pytest:}; expr=${expr//_or_/ or }
        timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "$expr" \
            > "$out/pytest_sel.log" 2>&1
        rc=$?; echo "pytest rc=$rc"; tail -5 "$out/pytest_sel.log"; fatal $rc && exit $rc ;;
    testsv:*)  # testsv:<variant> -> the GPU tests against variants/libsnappy_amd_<variant>.so (the CLI keeps the main library)
        v=${step#testsv:}
        SNAPPY_AMD_LIB=$PWD/lightweight-snappy_amd/variants/libsnappy_amd_$v.so timeout -k 10 700 \
            python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > "$out/gpu_tests_$v.log" 2>&1
        rc=$?; echo "testsv $v rc=$rc"; tail -3 "$out/gpu_tests_$v.log"; fatal $rc && exit $rc ;;
    e2e:*)  # e2e:<total bytes> -> end-to-end pipeline over a 1-rank RCCL communicator, overlapped vs serialised, twice
        tb=${step#e2e:}
        for r in 1 2; do for o in "" "--no-e2e-overlap"; do
            timeout -k 10 400 python -u bench.py --dist-world1 --total-bytes $tb --steps 2 --warmup 1 --e2e-steps 2 \
                --no-sub --no-cpu-baseline --no-host-e2e $o >> "$out/e2e_$tb.json" 2>> "$out/e2e_$tb.err"
            rc=$?; echo "e2e '$o' rc=$rc"; [ $rc -ne 0 ] && exit $rc
        done; done
        python3 -c "import json,sys; [print(d['ms_per_step'], d['value'], d['value_end_to_end'], d['exchange']['end_to_end_ms_per_step'], d['exchange']['end_to_end_step'][-40:], d['round_trip_ok']) for d in map(json.loads, [l for l in open(sys.argv[1]) if l.startswith('{')])]" "$out/e2e_$tb.json" ;;
    rst:*)  # rst:<chunk> -> K1r / K1r64 refresh share with the asm loop (SNAPPY_K1R_RSTAMPS build, variant rst), 256 MiB
        IFS=: read -r _ chunk <<< "$step"
        timeout -k 10 200 python -u tools/k1r_rstamps.py 268435456 $chunk rst > "$out/rst_$chunk.log" 2>&1
        rc=$?; echo "rst rc=$rc"; cat "$out/rst_$chunk.log"; [ $rc -ne 0 ] && exit $rc ;;
    prof1m)  # configs[0]'s 1,000,000-byte compress alone: K1r64 over 16 blocks = one lone wave's chain
        timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$out/prof1m" -o run --output-format csv -- \
            python3 tools/run_once.py T 1000000 65536 > "$out/prof1m.log" 2>&1
        rc=$?; echo "prof1m rc=$rc"; [ $rc -ne 0 ] && exit $rc ;;
    tracee2e)  # kernel trace of the end-to-end pipeline over a 1-rank RCCL communicator (C2 beside K1r?)
        timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$out/tracee2e" -o run --output-format csv -- \
            python3 bench.py --dist-world1 --dist-backend nccl --total-bytes 8589934592 --steps 1 --warmup 1 \
            --e2e-steps 1 --no-sub --no-cpu-baseline --no-host-e2e > "$out/tracee2e.log" 2>&1
        rc=$?; echo "tracee2e rc=$rc"; [ $rc -ne 0 ] && exit $rc ;;
    *) echo "unknown step $step"; exit 2 ;;
    esac
done
echo "[$(date +%T)] done"
