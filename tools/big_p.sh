#!/bin/bash
set -o pipefail
OUT=gpurun_out/big_p
mkdir -p $OUT
for w in fedavg iterative weighted; do
  timeout -k 10 300 python tools/ab_variants.py --workload $w --rounds 6 --variants 6,11,12,13,14,0 > $OUT/$w.json 2>>$OUT/err.log || exit 1
done
python3 -c "
import json,glob
for f in sorted(glob.glob('$OUT/*.json')):
    d=json.load(open(f)); print(d['workload'], d['P'], d['N'], {k:v['GBps_median'] for k,v in d['variants'].items()})
"
