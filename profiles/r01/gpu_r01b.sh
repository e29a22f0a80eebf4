#!/bin/bash
# GPU tests + every bench workload (one MI355X).
set -o pipefail
OUT=gpurun_out/r01b
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $OUT/gpu_tests.log
[ $rc -le 1 ] || exit $rc
for w in resnet18-fedavg resnet18-iterative resnet18-weighted mnist-state; do
  timeout -k 10 200 python bench.py --workload $w --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { echo "bench $w rc=$?"; tail -3 $OUT/bench_$w.err; exit 1; }
done
timeout -k 10 200 python bench.py --workload resnet18-secagg --steps 10 --warmup 2 > $OUT/bench_resnet18-secagg.json 2> $OUT/bench_resnet18-secagg.err || { echo "secagg rc=$?"; tail -3 $OUT/bench_resnet18-secagg.err; }
timeout -k 10 300 python bench.py --workload c4-stream --steps 4 --warmup 1 > $OUT/bench_c4-stream.json 2> $OUT/bench_c4-stream.err || { echo "c4 rc=$?"; tail -3 $OUT/bench_c4-stream.err; exit 1; }
timeout -k 10 300 python bench.py --workload c5-ingest --steps 3 --warmup 1 > $OUT/bench_c5-ingest.json 2> $OUT/bench_c5-ingest.err || { echo "c5 rc=$?"; tail -3 $OUT/bench_c5-ingest.err; exit 1; }
echo done
