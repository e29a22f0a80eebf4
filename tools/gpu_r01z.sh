#!/bin/bash
# Share-State ingest: tests after the SSE2 stats pass, then the pinned fill size sweep.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r01z
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_shares.py -x -q --timeout 120 --timeout-method thread > $OUT/shares_tests.log 2>&1
rc=$?; tail -2 $OUT/shares_tests.log; [ $rc -eq 0 ] || exit $rc
for mb in 8 16 32 128; do
  PGH_SHARE_FILL_MB=$mb timeout -k 10 300 python bench.py --workload resnet18-secagg-state --steps 3 --warmup 1 --no-cpu-baseline > $OUT/fill_$mb.json 2> $OUT/fill_$mb.err || exit $?
  python -c "import json;r=json.loads(open('$OUT/fill_$mb.json').read());print($mb, r['value'], r['wire_GBps'], r['h2d_GBps'], r['ms_per_step'])"
done
echo done
