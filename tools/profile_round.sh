#!/bin/bash
# Evidence pass on one MI355X: GPU tests, smoke, every bench workload, rocprofv3 --stats of the
# default bench, HBM PMC passes (separate FETCH_SIZE / WRITE_SIZE runs) for the resident kernels,
# host base64 rate.   usage: bash tools/profile_round.sh <tag>   (writes gpurun_out/<tag>/)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-round}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
for w in resnet18-iterative resnet18-weighted resnet18-secagg mnist-state secagg-clients; do
  timeout -k 10 200 python bench.py --workload $w --steps 10 --warmup 2 > $OUT/bench_$w.json 2> $OUT/bench_$w.err || exit $?
done
timeout -k 10 300 python bench.py --workload resnet18-state --steps 3 --warmup 1 > $OUT/bench_resnet18-state.json 2> $OUT/bench_resnet18-state.err || exit $?
timeout -k 10 300 python bench.py --workload resnet18-report --steps 3 --warmup 1 > $OUT/bench_resnet18-report.json 2> $OUT/bench_resnet18-report.err || exit $?
timeout -k 10 400 python bench.py --workload resnet18-secagg-state --steps 3 --warmup 1 > $OUT/bench_resnet18-secagg-state.json 2> $OUT/bench_resnet18-secagg-state.err || exit $?
timeout -k 10 300 python bench.py --workload c4-stream --steps 4 --warmup 1 > $OUT/bench_c4-stream.json 2> $OUT/bench_c4-stream.err || exit $?
timeout -k 10 300 python bench.py --workload c5-ingest --steps 3 --warmup 1 > $OUT/bench_c5-ingest.json 2> $OUT/bench_c5-ingest.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 > $OUT/bench_resnet18-fedavg.json 2> $OUT/bench_trace.err || exit $?
for w in resnet18-iterative resnet18-secagg; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_$w -o run --output-format csv -- python3 bench.py --workload $w --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_trace_$w.json 2> $OUT/bench_trace_$w.err || exit $?
done
for w in resnet18-fedavg resnet18-iterative resnet18-weighted resnet18-secagg; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 200 rocprofv3 --pmc $c -d $OUT/pmc_${w}_$c -o run --output-format csv -- python3 bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > $OUT/pmc_${w}_$c.log 2>&1 || exit $?
  done
done
timeout -k 10 200 python tools/bench_b64.py > $OUT/b64.log 2>&1 || exit $?
echo done
