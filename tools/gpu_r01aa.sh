#!/bin/bash
# Atomic multi-party share ingest: share tests, whole GPU suite, secagg-state bench line.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r01aa
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_shares.py -x -q --timeout 120 --timeout-method thread > $OUT/shares_tests.log 2>&1
rc=$?; tail -2 $OUT/shares_tests.log; [ $rc -eq 0 ] || { tail -40 $OUT/shares_tests.log; exit $rc; }
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --workload resnet18-secagg-state --steps 3 --warmup 1 > $OUT/bench_resnet18-secagg-state.json 2> $OUT/bench_resnet18-secagg-state.err || exit $?
python -c "import json;r=json.loads(open('$OUT/bench_resnet18-secagg-state.json').read());print(r['value'], r['wire_GBps'], r['ms_per_step'], r['cpu_baseline']['cycle_close_ms_per_client'])"
echo done
