#!/bin/bash
set -o pipefail
OUT=gpurun_out/small_p2
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit 1
for cfg in "50000 60000" "100000 30000" "311650 10000" "1000000 3000" "3000000 1000" "11689512 300"; do
  set -- $cfg
  timeout -k 10 200 python tools/ab_variants.py --workload fedavg --params $1 --clients $2 --rounds 3 --variants 6,10,11,12,13,14 > $OUT/fedavg_p$1.json 2>>$OUT/err.log || exit 1
done
python3 -c "
import json,glob
for f in sorted(glob.glob('$OUT/fedavg_p*.json')):
    d=json.load(open(f)); print(d['P'], {k:v['GBps_median'] for k,v in d['variants'].items()})
"
