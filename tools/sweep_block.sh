#!/bin/bash
# Block width sweep (PGH_BLOCK_BYTES) x variant on the ResNet-18 fold and the secagg share sum.
set -o pipefail
OUT=gpurun_out/sweep_block
mkdir -p $OUT
for bb in 16384 65536 262144 1048576 4194304; do
  PGH_BLOCK_BYTES=$bb timeout -k 10 200 python tools/ab_variants.py --workload fedavg --rounds 4 --variants 0,6,15,11 > $OUT/fedavg_bb$bb.json 2>>$OUT/err.log || exit 1
  PGH_BLOCK_BYTES=$bb timeout -k 10 300 python tools/ab_variants.py --workload secagg --rounds 3 --variants 14,16,12 > $OUT/secagg_bb$bb.json 2>>$OUT/err.log || exit 1
done
python3 -c "
import json,glob
for f in sorted(glob.glob('$OUT/*.json')):
    d=json.load(open(f)); print(f.split('/')[-1], {k:v['GBps_median'] for k,v in d['variants'].items()})
"
