#!/bin/bash
# Non-temporal staging copies (PGH_NT_COPY) A/B on the host-bound bytes -> bytes paths.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r01ab
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for nt in 0 1; do
    for w in resnet18-state resnet18-secagg-state; do
      PGH_NT_COPY=$nt timeout -k 10 300 python bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > $OUT/${w}_nt${nt}_r$rep.json 2> $OUT/${w}_nt${nt}_r$rep.err || exit $?
      python -c "import json;r=json.loads(open('$OUT/${w}_nt${nt}_r$rep.json').read());print('$w nt=$nt', r['value'], r.get('wire_GBps'), r.get('h2d_GBps'), r['ms_per_step'])"
    done
  done
done
PGH_NT_COPY=1 timeout -k 10 120 python tools/time_mnist_state.py > $OUT/time_mnist_nt1.log 2>&1 || exit $?
PGH_NT_COPY=0 timeout -k 10 120 python tools/time_mnist_state.py > $OUT/time_mnist_nt0.log 2>&1 || exit $?
tail -1 $OUT/time_mnist_nt1.log; tail -1 $OUT/time_mnist_nt0.log
echo done
