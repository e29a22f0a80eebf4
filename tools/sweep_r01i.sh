#!/bin/bash
set -o pipefail
OUT=gpurun_out/sweep_r01i
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit 1
for w in fedavg iterative; do
  timeout -k 10 300 python tools/ab_variants.py --workload $w --rounds 6 --variants 11,12,14,15,16,17,18 > $OUT/$w.json 2>>$OUT/err.log || exit 1
done
timeout -k 10 300 python tools/ab_variants.py --workload secagg --clients 250 --rounds 6 --variants 6,11,12,14,15,16,17,18 > $OUT/secagg.json 2>>$OUT/err.log || exit 1
timeout -k 10 300 python tools/ab_variants.py --workload secagg --clients 2500 --params 311650 --rounds 4 --variants 6,11,12,14,15,16,17,18 > $OUT/secagg_small.json 2>>$OUT/err.log || exit 1
timeout -k 10 300 python tools/ab_variants.py --workload fedavg --clients 60000 --params 50000 --rounds 4 --variants 14,16,17,18 > $OUT/fedavg_50k.json 2>>$OUT/err.log || exit 1
python3 -c "
import json,glob
for f in sorted(glob.glob('$OUT/*.json')):
    d=json.load(open(f)); print(d['workload'], d['P'], d['N'], {k:v['GBps_median'] for k,v in d['variants'].items()})
"
