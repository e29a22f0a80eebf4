#!/bin/bash
# Engine warm-up at pgh_create: first closes from a fresh Engine with and without it, then all
# GPU tests and smoke on HEAD.
set -o pipefail
OUT=gpurun_out/r01an
mkdir -p $OUT
PGH_WARMUP=0 timeout -k 10 120 python tools/time_mnist_cold.py > $OUT/mnist_cold_warmup0.log 2>&1 || exit $?
timeout -k 10 120 python tools/time_mnist_cold.py > $OUT/mnist_cold_warmup1.log 2>&1 || exit $?
timeout -k 10 120 python tools/time_mnist_first.py > $OUT/mnist_first_warmup1.log 2>&1 || exit $?
cat $OUT/mnist_cold_warmup0.log $OUT/mnist_cold_warmup1.log $OUT/mnist_first_warmup1.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -20 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
