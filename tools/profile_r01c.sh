#!/bin/bash
# Variant sweep + nt-default rocprofv3 stats and HBM PMC passes (one MI355X).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/prof_r01c
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ab_variants.py --workload fedavg --rounds 6 > $OUT/ab_fedavg.json 2> $OUT/ab_fedavg.err || exit $?
timeout -k 10 300 python tools/ab_variants.py --workload iterative --rounds 4 > $OUT/ab_iterative.json 2> $OUT/ab_iterative.err || exit $?
timeout -k 10 300 python tools/ab_variants.py --workload secagg --clients 250 --rounds 4 --variants 0,2,4,6,7 > $OUT/ab_secagg.json 2> $OUT/ab_secagg.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 > $OUT/bench_trace.json 2> $OUT/bench_trace.err || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $c -d $OUT/pmc_$c -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $OUT/pmc_$c.log 2>&1 || exit $?
  timeout -s KILL 150 rocprofv3 --pmc $c -d $OUT/pmc_secagg_$c -o run --output-format csv -- python3 bench.py --workload resnet18-secagg --clients 250 --steps 3 --warmup 1 > $OUT/pmc_secagg_$c.log 2>&1 || exit $?
  timeout -s KILL 150 rocprofv3 --pmc $c -d $OUT/pmc_iter_$c -o run --output-format csv -- python3 bench.py --workload resnet18-iterative --steps 3 --warmup 1 > $OUT/pmc_iter_$c.log 2>&1 || exit $?
done
echo done
