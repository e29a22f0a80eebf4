#!/bin/bash
# CPU baselines beside the non-resident bench lines (c4/c5 extrapolated from a client sample, the
# bytes -> bytes lines against oracle.cycle_close_state_torch) + MNIST per-call breakdown.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r01v
mkdir -p $OUT
for w in mnist-state resnet18-state resnet18-report; do
  timeout -k 10 300 python bench.py --workload $w --steps 3 --warmup 1 > $OUT/bench_$w.json 2> $OUT/bench_$w.err || exit $?
done
timeout -k 10 300 python bench.py --workload c4-stream --steps 3 --warmup 1 > $OUT/bench_c4-stream.json 2> $OUT/bench_c4-stream.err || exit $?
timeout -k 10 300 python bench.py --workload c5-ingest --steps 3 --warmup 1 > $OUT/bench_c5-ingest.json 2> $OUT/bench_c5-ingest.err || exit $?
timeout -k 10 300 python bench.py --workload secagg-clients --steps 5 --warmup 1 > $OUT/bench_secagg-clients.json 2> $OUT/bench_secagg-clients.err || exit $?
timeout -k 10 120 python tools/time_mnist_state.py > $OUT/time_mnist_state.log 2>&1 || exit $?
echo done
