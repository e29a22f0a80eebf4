#!/bin/bash
# Secagg shares as State bytes (GPU varint decode): new GPU tests first, then the whole suite,
# then the resnet18-secagg-state bench line and a rocprof stats pass of it.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r01y
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_shares.py -x -v --timeout 120 --timeout-method thread > $OUT/shares_tests.log 2>&1
rc=$?; tail -25 $OUT/shares_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --workload resnet18-secagg-state --steps 3 --warmup 1 > $OUT/bench_resnet18-secagg-state.json 2> $OUT/bench_resnet18-secagg-state.err || exit $?
cat $OUT/bench_resnet18-secagg-state.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace_secagg_state -o run --output-format csv -- python3 bench.py --workload resnet18-secagg-state --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench_trace_secagg_state.json 2> $OUT/bench_trace_secagg_state.err || exit $?
echo done
