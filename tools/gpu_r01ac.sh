#!/bin/bash
# D2H piece size (PGH_D2H_PIECE_MB) A/B on the report-time close (47 MB checkpoint patched from HBM).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r01ac
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "patch or ckpt or incremental or state" > $OUT/gpu_tests.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for mb in 0 4 8 16; do
    PGH_D2H_PIECE_MB=$mb timeout -k 10 300 python bench.py --workload resnet18-report --steps 4 --warmup 1 --no-cpu-baseline > $OUT/report_p${mb}_r$rep.json 2> $OUT/report_p${mb}_r$rep.err || exit $?
    python -c "import json;r=json.loads(open('$OUT/report_p${mb}_r$rep.json').read());print('piece', $mb, r['close_ms_after_last_report'], r['close_ms_after_last_report_all'])"
  done
done
echo done
