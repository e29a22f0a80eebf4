#!/bin/bash
# Masked last row batch (r01p): parity, then the default variants at big / small shards, odd N.
set -o pipefail
OUT=gpurun_out/ab_tail
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?; tail -3 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for w in fedavg iterative weighted; do timeout -k 10 300 python tools/ab_variants.py --workload $w --rounds 4 --variants 0,15,11 > $OUT/$w.json 2>>$OUT/err.log || exit 1; done
timeout -k 10 300 python tools/ab_variants.py --workload secagg --rounds 3 --variants 14,16 > $OUT/secagg.json 2>>$OUT/err.log || exit 1
for cfg in "100000 30000" "311650 10000" "1000000 3000"; do set -- $cfg
  for w in fedavg iterative; do timeout -k 10 200 python tools/ab_variants.py --workload $w --params $1 --clients $2 --rounds 3 --variants 0,11,14,17 > $OUT/${w}_p$1.json 2>>$OUT/err.log || exit 1; done; done
python3 -c "
import json,glob
for f in sorted(glob.glob('$OUT/*.json')):
    d=json.load(open(f)); print(d['workload'], d['P'], d['N'], {k:v['GBps_median'] for k,v in d['variants'].items()})
"
