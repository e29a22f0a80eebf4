#!/bin/bash
# Round-1 measurement pass on one MI355X: variant A/B, kernel trace + stats, HBM PMC passes.
# Usage (from the repo root, on the GPU box): bash tools/profile_r01.sh
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/prof_r01
mkdir -p $OUT
timeout -k 10 300 python tools/ab_variants.py --workload fedavg > $OUT/ab_fedavg.json 2> $OUT/ab_fedavg.err || exit $?
timeout -k 10 300 python tools/ab_variants.py --workload iterative > $OUT/ab_iterative.json 2> $OUT/ab_iterative.err || exit $?
timeout -k 10 300 python tools/ab_variants.py --workload secagg --clients 250 > $OUT/ab_secagg.json 2> $OUT/ab_secagg.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_trace.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $OUT/pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $OUT/pmc_write.log 2>&1 || exit $?
echo done
