#!/bin/bash
# Whole GPU suite (incl. pipelined variants 21/22 and the overlapped checkpoint patch), then the
# MNIST per-call breakdown and the bytes -> bytes bench lines.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r01x
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $OUT/gpu_tests.log | head -20; exit $rc; }
timeout -k 10 120 python tools/time_mnist_state.py > $OUT/time_mnist_state.log 2>&1 || exit $?
cat $OUT/time_mnist_state.log
timeout -k 10 200 python bench.py --workload mnist-state --steps 20 --warmup 3 > $OUT/bench_mnist-state.json 2> $OUT/bench_mnist-state.err || exit $?
timeout -k 10 300 python bench.py --workload resnet18-report --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_resnet18-report.json 2> $OUT/bench_resnet18-report.err || exit $?
timeout -k 10 300 python bench.py --workload resnet18-state --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_resnet18-state.json 2> $OUT/bench_resnet18-state.err || exit $?
echo done
