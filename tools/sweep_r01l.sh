#!/bin/bash
# Variant sweep on the column-blocked slab (r01l): big / mid / small shards, every mode.
set -o pipefail
OUT=gpurun_out/sweep_r01l
mkdir -p $OUT
for w in fedavg iterative weighted; do
  timeout -k 10 300 python tools/ab_variants.py --workload $w --rounds 5 --variants 0,6,7,8,9,10,11,15,14 > $OUT/$w.json 2>>$OUT/err.log || exit 1
done
timeout -k 10 400 python tools/ab_variants.py --workload secagg --rounds 4 --variants 0,6,11,12,14,15,16,18 > $OUT/secagg.json 2>>$OUT/err.log || exit 1
timeout -k 10 300 python tools/ab_variants.py --workload secagg --clients 2500 --params 311650 --rounds 4 --variants 0,6,11,12,14,15 > $OUT/secagg_small.json 2>>$OUT/err.log || exit 1
for cfg in "100000 30000" "311650 10000" "1000000 3000" "3000000 1000"; do
  set -- $cfg
  timeout -k 10 200 python tools/ab_variants.py --workload fedavg --params $1 --clients $2 --rounds 3 --variants 0,6,11,12,14,15 > $OUT/fedavg_p$1.json 2>>$OUT/err.log || exit 1
  timeout -k 10 200 python tools/ab_variants.py --workload iterative --params $1 --clients $2 --rounds 3 --variants 0,6,11,12,14,15 > $OUT/iterative_p$1.json 2>>$OUT/err.log || exit 1
done
python3 -c "
import json,glob
for f in sorted(glob.glob('$OUT/*.json')):
    d=json.load(open(f)); print(d['workload'], d['P'], d['N'], {k:v['GBps_median'] for k,v in d['variants'].items()})
"
