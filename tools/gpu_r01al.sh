#!/bin/bash
# Confirm HEAD (8 MiB D2H pieces + parallel pre-fault by default): all GPU tests, smoke, the
# bytes-path bench lines and the default bench.
set -o pipefail
OUT=gpurun_out/r01al
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -20 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
for w in resnet18-report resnet18-state mnist-state resnet18-secagg-state; do
  timeout -k 10 400 python bench.py --workload $w --steps 3 --warmup 1 > $OUT/bench_$w.json 2> $OUT/bench_$w.err || exit $?
done
timeout -k 10 300 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || exit $?
echo done
