#!/bin/bash
# Auto-variant profile (r01g): tests, state benches, rocprofv3 stats + HBM PMC passes per workload.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/prof_r01g
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for w in mnist-state resnet18-iterative resnet18-weighted resnet18-secagg; do timeout -k 10 200 python bench.py --workload $w --steps 10 --warmup 2 > $OUT/bench_$w.json 2> $OUT/bench_$w.err || exit $?; done
timeout -k 10 300 python bench.py --workload resnet18-state --steps 3 --warmup 1 > $OUT/bench_resnet18-state.json 2> $OUT/bench_resnet18-state.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 > $OUT/bench_trace.json 2> $OUT/bench_trace.err || exit $?
for w in resnet18-fedavg resnet18-iterative resnet18-weighted resnet18-secagg; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 200 rocprofv3 --pmc $c -d $OUT/pmc_${w}_$c -o run --output-format csv -- python3 bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > $OUT/pmc_${w}_$c.log 2>&1 || exit $?
  done
done
echo done
