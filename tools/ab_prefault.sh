#!/bin/bash
# A/B of PGH_PREFAULT (parallel pre-fault of the fresh checkpoint bytes during the fold + D2H):
# State-bytes close phases, report-time close, MNIST close; then the GPU tests that touch the patch.
set -o pipefail
OUT=gpurun_out/r01aj
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "state or incremental or report or ckpt" > $OUT/gpu_tests.log 2>&1 || { tail -20 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
for r in 1 2; do
  for pf in 0 1; do
    PGH_PREFAULT=$pf timeout -k 10 200 python tools/time_resnet_state.py > $OUT/phases_pf${pf}_r$r.log 2>&1 || exit $?
    PGH_PREFAULT=$pf timeout -k 10 300 python bench.py --workload resnet18-report --steps 3 --warmup 1 --no-cpu-baseline > $OUT/report_pf${pf}_r$r.json 2> $OUT/report_pf${pf}_r$r.err || exit $?
    PGH_PREFAULT=$pf timeout -k 10 200 python bench.py --workload mnist-state --steps 20 --warmup 3 --no-cpu-baseline > $OUT/mnist_pf${pf}_r$r.json 2> $OUT/mnist_pf${pf}_r$r.err || exit $?
    echo "pf=$pf r=$r: $(tail -1 $OUT/phases_pf${pf}_r$r.log)"
  done
done
echo done
