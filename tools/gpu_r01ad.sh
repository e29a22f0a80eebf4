#!/bin/bash
# Row-skew experiment on the column-blocked slab: rows of a block 2^k + skew elements apart.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r01ad
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
PGH_ROW_SKEW=256 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shares.py tests/test_gpu_stream.py -x -q --timeout 120 --timeout-method thread -k "mid_size or synthetic_sampled or share_state or ring or stream" > $OUT/skew_tests.log 2>&1
rc=$?; tail -2 $OUT/skew_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/skew_tests.log | head; }
for rep in 1 2; do
  for sk in 0 64 256 1024; do
    for w in resnet18-fedavg resnet18-secagg; do
      PGH_ROW_SKEW=$sk timeout -k 10 200 python bench.py --workload $w --steps 10 --warmup 2 --no-cpu-baseline > $OUT/${w}_s${sk}_r$rep.json 2> $OUT/${w}_s${sk}_r$rep.err || exit $?
      python -c "import json;r=json.loads(open('$OUT/${w}_s${sk}_r$rep.json').read());print('$w skew=$sk', r['value'], r['roofline']['achieved'], r['roofline']['kernel_ms_avg'])"
    done
  done
done
echo done
