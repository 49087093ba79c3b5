# K5p A/B on the GPU box: the index GPU tests, then tools/k5_time.py (text and random, 256 MiB) for the tree library and variants/libsnappy_amd_prev.so (tools/build_prev.sh HEAD prev), 3 interleaved rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "index or foreign or xblock or reference_stream or errors" > gpurun_out/k5ab_tests.log 2>&1 || exit $?
for r in 1 2 3; do
  for v in default prev; do
    lib=""; [ $v != default ] && lib=$PWD/lightweight-snappy_amd/variants/libsnappy_amd_$v.so
    for kind in T R; do
      SNAPPY_AMD_LIB=$lib timeout -k 10 120 python -u tools/k5_time.py $kind 268435456 5 > gpurun_out/k5ab_${v}_${kind}_$r.log 2>&1 || exit $?
      echo "$v $kind $r: $(tail -1 gpurun_out/k5ab_${v}_${kind}_$r.log)"
    done
  done
done
